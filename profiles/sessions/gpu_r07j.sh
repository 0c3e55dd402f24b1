#!/bin/bash
# Round 5: device-driven pair levels against round 4's per-level host synchronisation, fractal.scene 1080p.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r07k}
H=tinyraytracerinrust_amd/build/librt_mi355x_head.so
for R in 1; do
  RT_LIB_PATH=$H timeout -k 10 300 python -u tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1 7 >> $O/${T}_fractal.txt 2>&1 || { tail $O/${T}_fractal.txt; exit 1; }
  echo "^ round-4 (per-level synchronisation)" >> $O/${T}_fractal.txt
  timeout -k 10 300 python -u tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1 7 >> $O/${T}_fractal.txt 2>&1 || { tail $O/${T}_fractal.txt; exit 1; }
  echo "^ device-driven levels" >> $O/${T}_fractal.txt
done
grep -v amdgpu.ids $O/${T}_fractal.txt
RT_LIB_PATH=$H timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_kt_head -o run -- python3 tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1 3 > /dev/null 2>&1 || { echo kt head failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_kt_new -o run -- python3 tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1 3 > /dev/null 2>&1 || { echo kt new failed; exit 1; }
echo session done
