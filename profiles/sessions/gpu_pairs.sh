#!/bin/bash
# Round-3 pair-path session: wavefront GPU tests, fractal / other scenes timed per pairs mode, then
# (optionally) a rocprofv3 kernel trace of one fractal wavefront frame.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r03x}
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_wavefront.py -x -q --timeout 120 --timeout-method thread > $O/${T}_wf_tests.txt 2>&1 || { tail -40 $O/${T}_wf_tests.txt; exit 1; }
  tail -2 $O/${T}_wf_tests.txt
fi
timeout -k 10 300 python -u tools/scene_timing.py fractal 1920x1080 0 10 mega,wavefront:p0,wavefront:p1,wavefront:p2 5 > $O/${T}_fractal_timing.txt 2>&1 || { tail $O/${T}_fractal_timing.txt; exit 1; }
cat $O/${T}_fractal_timing.txt
timeout -k 10 300 python -u tools/scene_timing.py spinning_globes 1920x1080 0.3 10 mega,wavefront:p0,wavefront:p1,wavefront:p2 5 > $O/${T}_sg_timing.txt 2>&1 || { tail $O/${T}_sg_timing.txt; exit 1; }
cat $O/${T}_sg_timing.txt
timeout -k 10 300 python -u tools/scene_timing.py globes 1920x1080 0 5 auto,wavefront:p0,wavefront:p1,wavefront:p2 5 > $O/${T}_g_timing.txt 2>&1 || { tail $O/${T}_g_timing.txt; exit 1; }
cat $O/${T}_g_timing.txt
if [ "${KT:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_kt -o run -- python3 tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1 2 > $O/${T}_kt.txt 2> $O/${T}_kt.err || { tail $O/${T}_kt.err; exit 1; }
fi
echo session done
