#!/bin/bash
# Round 5 final consolidation at HEAD: the GPU suite, every config's bench line, PMC passes of all four
# configs, the headline kernel trace, the fractal timing and a 2-rank rehearsal of the N > 1 path.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r08m}
TAG=$T bash tools/gpu_final.sh || exit 1
TAG=$T bash tools/gpu_pmc_configs.sh || exit 1
timeout -k 10 300 python -u tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1 7 2>&1 | grep -v amdgpu.ids > $O/${T}_fractal.txt || exit 1
cat $O/${T}_fractal.txt
timeout -k 10 300 python bench.py --gpus 2 --rehearse-one-gpu --steps 5 --warmup 2 > $O/${T}_rehearse2.json 2> $O/${T}_rehearse2.err || { tail $O/${T}_rehearse2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/${T}_rehearse2.json'));print('rehearse 2', d.get('value'), d.get('ms_per_step'), d.get('frame_check'))"
echo consolidation done
