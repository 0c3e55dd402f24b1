#!/bin/bash
# Round 5: pair-buffer size (RT_WFP_BUF 256 / 1024) and candidate workgroup waves (2 / 8) against the product, fractal.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r08l}
B=tinyraytracerinrust_amd/build
for R in 1 2; do
  for L in tinyraytracerinrust_amd/librt_mi355x.so $B/librt_mi355x_b256.so $B/librt_mi355x_b1024.so $B/librt_mi355x_cw2.so $B/librt_mi355x_cw8.so; do
    RT_LIB_PATH=$L timeout -k 10 300 python -u tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1 7 2>&1 | grep -v amdgpu.ids | sed "s|\$| [$(basename $L)]|" >> $O/${T}_fractal.txt || exit 1
  done
done
cat $O/${T}_fractal.txt
echo session done
