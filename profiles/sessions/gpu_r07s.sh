#!/bin/bash
# Round 5: chunked bucket-sort histogram against the previous library, fractal.scene 1080p d10.
# pair path from level 0 (p2) for reference.  fractal.scene 1080p d10.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r07s}
B=tinyraytracerinrust_amd/build
P=tinyraytracerinrust_amd/librt_mi355x.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_wavefront.py -x -q --timeout 300 --timeout-method thread > $O/${T}_pytest_wf.txt 2>&1 || { tail -40 $O/${T}_pytest_wf.txt; exit 1; }
tail -2 $O/${T}_pytest_wf.txt
for R in 1 2; do
  for L in $B/librt_mi355x_prev.so $P; do
    RT_LIB_PATH=$L timeout -k 10 300 python -u tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1 7 2>&1 | grep -v amdgpu.ids | sed "s|\$| [$(basename $L)]|" >> $O/${T}_fractal.txt || { tail $O/${T}_fractal.txt; exit 1; }
  done
done
cat $O/${T}_fractal.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_kt -o run -- python3 tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1 3 > /dev/null 2>&1 || { echo kt failed; exit 1; }
echo session done
