#!/bin/bash
# Round 5: pair-path launches per level cut (level check and resets folded into the shading kernel,
# bucket-sort scan fused into the scatter, occupancy-sized candidate grids): wavefront tests, fractal
# timing against the previous library, per-level counts (diag build), kernel trace; the quad-order
# diagnostic on the 1080p sphere.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r07o}
P=tinyraytracerinrust_amd/librt_mi355x.so
V=tinyraytracerinrust_amd/build/librt_mi355x_prev.so
D=tinyraytracerinrust_amd/build/librt_mi355x_wfdbg.so
Q=tinyraytracerinrust_amd/build/librt_mi355x_quad.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_wavefront.py -x -q --timeout 300 --timeout-method thread > $O/${T}_pytest_wf.txt 2>&1 || { tail -40 $O/${T}_pytest_wf.txt; exit 1; }
tail -2 $O/${T}_pytest_wf.txt
for R in 1 2; do
  RT_LIB_PATH=$V timeout -k 10 300 python -u tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1 7 >> $O/${T}_fractal.txt 2>&1 || { tail $O/${T}_fractal.txt; exit 1; }
  echo "^ previous library" >> $O/${T}_fractal.txt
  timeout -k 10 300 python -u tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1 7 >> $O/${T}_fractal.txt 2>&1 || { tail $O/${T}_fractal.txt; exit 1; }
  echo "^ fewer launches per level" >> $O/${T}_fractal.txt
done
grep -v amdgpu.ids $O/${T}_fractal.txt
RT_LIB_PATH=$D RT_WF_DEBUG=1 timeout -k 10 300 python -u tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1 2 > $O/${T}_levels.txt 2>&1 || { tail $O/${T}_levels.txt; exit 1; }
grep -v amdgpu.ids $O/${T}_levels.txt | tail -3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_kt -o run -- python3 tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1 3 > /dev/null 2>&1 || { echo kt failed; exit 1; }
timeout -k 10 300 python -u tools/ab_libs.py $P $Q --config sphere1080d0 > $O/${T}_quad_ab.txt 2>&1 || { tail -20 $O/${T}_quad_ab.txt; exit 1; }
timeout -k 10 300 python -u tools/ab_libs.py $P $Q --config globes1080d5 >> $O/${T}_quad_ab.txt 2>&1 || { tail -20 $O/${T}_quad_ab.txt; exit 1; }
grep -v amdgpu.ids $O/${T}_quad_ab.txt
echo session done
