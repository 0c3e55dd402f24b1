#!/bin/bash
# Round 5: cached frame stores for primary-ray launches (k_rows.hip RT_CACHED_FRAME_BYTES) -- A/B
# against the previous product (b9114232) on the three row configs, then the round-end session at
# this binary (GPU suite, bench lines, headline / anim PMC passes, kernel trace: tools/gpu_final.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r08s}
P=tinyraytracerinrust_amd/librt_mi355x.so
V=tinyraytracerinrust_amd/build/librt_mi355x_prev.so
for C in globes4k globes1080d5 sphere1080d0; do
  timeout -k 10 300 python -u tools/ab_libs.py $V $P --config $C >> $O/${T}_cached_ab.txt 2>&1 || { tail -20 $O/${T}_cached_ab.txt; exit 1; }
done
cat $O/${T}_cached_ab.txt
TAG=$T bash tools/gpu_final.sh || exit 1
echo part 1 done
