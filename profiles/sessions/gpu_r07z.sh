#!/bin/bash
# Round 5: anim120 over 1 / 2 / 3 / 4 streams at HEAD; fractal timing at HEAD (camera-term tables).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r07z}
for R in 1 2; do
  for S in 1 2 3 4; do
    timeout -k 10 300 python bench.py --config anim120 --steps 5 --warmup 1 --no-cpu-baseline --streams $S > $O/${T}_anim_s$S.json 2> $O/${T}_anim_s$S.err || { tail $O/${T}_anim_s$S.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${T}_anim_s$S.json'));print('round $R streams $S', d['value'], d['ms_per_step'])" | tee -a $O/${T}_anim_streams.txt
  done
done
timeout -k 10 300 python -u tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1 7 2>&1 | grep -v amdgpu.ids > $O/${T}_fractal.txt || exit 1
cat $O/${T}_fractal.txt
echo session done
