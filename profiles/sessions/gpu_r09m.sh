#!/bin/bash
# Round 6, session r09m: fractal with f64 culling in the generic kernels (diagnostic c64) against HEAD and
# the round-5 library, per-kernel traces.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r09m}
A=tinyraytracerinrust_amd/ab
for L in $A/librt_mi355x_cff8ab5a.so $A/librt_mi355x_c64.so tinyraytracerinrust_amd/librt_mi355x.so; do
  B=$(basename $L .so)
  RT_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_${B}_kt -o run -- python3 tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1 7 > $O/${T}_${B}.txt 2>&1 || { tail $O/${T}_${B}.txt; exit 1; }
  grep "ordered median" $O/${T}_${B}.txt
done
echo session done
