#!/bin/bash
# Round 5: hierarchy ranges allowed up to 8 / 16 grid passes (RT_WFP_RANGE_PASSES) against the product's 4, fractal.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r08k}
B=tinyraytracerinrust_amd/build
for R in 1 2 3; do
  for L in tinyraytracerinrust_amd/librt_mi355x.so $B/librt_mi355x_p8.so $B/librt_mi355x_p16.so; do
    RT_LIB_PATH=$L timeout -k 10 300 python -u tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1 7 2>&1 | grep -v amdgpu.ids | sed "s|\$| [$(basename $L)]|" >> $O/${T}_fractal.txt || exit 1
  done
done
cat $O/${T}_fractal.txt
echo session done
