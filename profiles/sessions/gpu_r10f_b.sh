#!/bin/bash
# Round 6 consolidation, part B, at the binary whose PMC summary part A committed: the GPU suite, every
# bench config's line (roofline blocks from profiles/pmc_summary.json), the solo kernel trace of the
# headline bench, fractal (pair path), a 2-rank rehearsal of the N > 1 path, and smoke().
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r10f}
sha256sum tinyraytracerinrust_amd/librt_mi355x.so | cut -c1-16 > $O/${T}_so_sha16.txt
( while sleep 50; do date +%T >> $O/${T}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_pytest_gpu.txt 2>&1 || { tail -40 $O/${T}_pytest_gpu.txt; exit 1; }
  tail -2 $O/${T}_pytest_gpu.txt
fi
timeout -k 10 300 python bench.py > $O/${T}_bench.json 2> $O/${T}_bench.err || { tail $O/${T}_bench.err; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/${T}_bench_s20.json 2> $O/${T}_bench_s20.err || { tail $O/${T}_bench_s20.err; exit 1; }
for C in sphere1080d0 globes1080d5 anim120; do
  F=""; [ $C = anim120 ] && F="--steps 3 --warmup 2"
  timeout -k 10 400 python bench.py --config $C $F > $O/${T}_bench_$C.json 2> $O/${T}_bench_$C.err || { tail $O/${T}_bench_$C.err; exit 1; }
done
for f in $O/${T}_bench*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', d.get('config_name'), d['value'], d['ms_per_step'], (r.get('executed_fp64') or {}).get('pmc_matches_binary'))"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_kt -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/${T}_bench_kt.json 2> $O/${T}_kt.err || { tail $O/${T}_kt.err; exit 1; }
head -3 $O/${T}_kt/run_kernel_stats.csv
timeout -k 10 300 python -u tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1 7 2>&1 | grep -v amdgpu.ids > $O/${T}_fractal.txt || exit 1
cat $O/${T}_fractal.txt
timeout -k 10 300 python bench.py --gpus 2 --rehearse-one-gpu --steps 5 --warmup 2 > $O/${T}_rehearse2.json 2> $O/${T}_rehearse2.err || { tail $O/${T}_rehearse2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/${T}_rehearse2.json'));print('rehearse 2', d.get('value'), d.get('ms_per_step'), d.get('frame_check'))"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.txt 2>&1 || { tail $O/${T}_smoke.txt; exit 1; }
tail -3 $O/${T}_smoke.txt

timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gpu_gui_rebuild.py > $O/${T}_gui_rebuild.txt 2>&1 || { tail -30 $O/${T}_gui_rebuild.txt; exit 1; }
grep -E "rebuil.*ms|passed" $O/${T}_gui_rebuild.txt | cut -c1-200
echo session done
