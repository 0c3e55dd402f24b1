#!/bin/bash
# Wavefront / pair path: the wavefront and stores tests, fractal / spinning_globes / globes timings
# under the wavefront kernels, a kernel trace of fractal.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r05za}
( while sleep 50; do date +%T >> $O/${T}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_wavefront.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_pytest.txt 2>&1 || { tail -40 $O/${T}_pytest.txt; exit 1; }
tail -2 $O/${T}_pytest.txt
timeout -k 10 300 python -u tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p0,wavefront:p1,wavefront:p2 5 > $O/${T}_fractal.txt 2>&1 || { tail $O/${T}_fractal.txt; exit 1; }
timeout -k 10 300 python -u tools/scene_timing.py spinning_globes 1920x1080 0.3 10 wavefront:p0,wavefront:p1 5 > $O/${T}_sg.txt 2>&1 || { tail $O/${T}_sg.txt; exit 1; }
grep -h median $O/${T}_fractal.txt $O/${T}_sg.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_kt -o run -- python3 tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1 2 > $O/${T}_kt.txt 2> $O/${T}_kt.err || { tail $O/${T}_kt.err; exit 1; }
echo session done
