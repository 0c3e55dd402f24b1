#!/bin/bash
# Round 6, session r09l: per-kernel times of the fractal wavefront frame, round-5 library vs HEAD
# (rocprofv3 kernel trace of tools/scene_timing.py), to find the kernel the f32-culling commit slowed.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r09l}
A=tinyraytracerinrust_amd/ab
for L in $A/librt_mi355x_cff8ab5a.so tinyraytracerinrust_amd/librt_mi355x.so; do
  B=$(basename $L .so)
  RT_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_${B}_kt -o run -- python3 tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1 7 > $O/${T}_${B}.txt 2>&1 || { tail $O/${T}_${B}.txt; exit 1; }
  grep -v amdgpu.ids $O/${T}_${B}.txt
done
echo session done
