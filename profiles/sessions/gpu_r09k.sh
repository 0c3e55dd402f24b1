#!/bin/bash
# Round 6, session r09k: which change moved fractal 1080p (wavefront pair path): the library at the
# round-5 commit and at each round-6 kernel commit, fractal timing twice each, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r09k}
A=tinyraytracerinrust_amd/ab
for rep in 1 2; do
  for L in $A/librt_mi355x_cff8ab5a.so $A/librt_mi355x_c881d104.so $A/librt_mi355x_cea5f79b.so $A/librt_mi355x_c69c79a8.so $A/librt_mi355x_z.so tinyraytracerinrust_amd/librt_mi355x.so; do
    RT_LIB_PATH=$L timeout -k 10 300 python -u tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1 7 2>&1 | grep -v amdgpu.ids | sed "s|\$| [$(basename $L)]|" >> $O/${T}_fractal.txt || exit 1
  done
done
cat $O/${T}_fractal.txt
echo session done
