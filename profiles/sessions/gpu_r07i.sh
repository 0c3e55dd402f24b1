#!/bin/bash
# Round 5: device-driven pair levels (wavefront tests, fractal timing), then the frame-pool A/B (r07h).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=r07i
timeout -k 10 900 python -u -m pytest tests/test_gpu_wavefront.py -x -q --timeout 300 --timeout-method thread > $O/${T}_pytest_wf.txt 2>&1 || { tail -40 $O/${T}_pytest_wf.txt; exit 1; }
tail -2 $O/${T}_pytest_wf.txt
timeout -k 10 300 python -u tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1,auto 7 > $O/${T}_fractal.txt 2>&1 || { tail -20 $O/${T}_fractal.txt; exit 1; }
cat $O/${T}_fractal.txt
TAG=r07h bash tools/gpu_r07h.sh
