#!/bin/bash
# Round 5, second half of the round-end session at the cached-store binary: PMC passes of the other
# configs, the fractal (pair path) timing and a 2-rank rehearsal of the N > 1 path.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r08s}
TAG=$T bash tools/gpu_pmc_configs.sh || exit 1
# the box's copy of profiles/pmc_summary.json takes these passes, so the bench lines below carry the
# roofline blocks of this binary (the committed summary is regenerated from the merged gpurun_out/)
python3 tools/pmc_summary.py ${T}_globes1080d5 globes1080d5 rt_spec_rows_00 > /dev/null || exit 1
python3 tools/pmc_summary.py ${T}_sphere1080d0 sphere1080d0 rt_spec_rows_00 > /dev/null || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/${T}_bench2.json 2> $O/${T}_bench2.err || { tail $O/${T}_bench2.err; exit 1; }
for C in sphere1080d0 globes1080d5 anim120; do
  F=""; [ $C = anim120 ] && F="--steps 3 --warmup 2"
  timeout -k 10 400 python bench.py --config $C $F > $O/${T}_bench2_$C.json 2> $O/${T}_bench2_$C.err || { tail $O/${T}_bench2_$C.err; exit 1; }
done
for f in $O/${T}_bench2*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', d.get('config_name'), d['value'], d['ms_per_step'], r.get('executed_fp64',{}).get('pmc_matches_binary'))"; done
timeout -k 10 300 python -u tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1 7 2>&1 | grep -v amdgpu.ids > $O/${T}_fractal.txt || exit 1
cat $O/${T}_fractal.txt
timeout -k 10 300 python bench.py --gpus 2 --rehearse-one-gpu --steps 5 --warmup 2 > $O/${T}_rehearse2.json 2> $O/${T}_rehearse2.err || { tail $O/${T}_rehearse2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/${T}_rehearse2.json'));print('rehearse 2', d.get('value'), d.get('ms_per_step'), d.get('frame_check'))"
echo part 2 done
