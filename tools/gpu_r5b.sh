#!/bin/bash
# Round-4 session b: GPU tests (incl. the specialised and tail kernels), the spec A/B at 4K, and the
# N = 8 / 4 single-frame shares with the tail kernel and specialisation on / off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; T=${TAG:-r05c}; mkdir -p $O
L=tinyraytracerinrust_amd/librt_mi355x.so
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread ${PYTEST_ARGS:-} > $O/${T}_pytest_gpu.txt 2>&1 || { tail -40 $O/${T}_pytest_gpu.txt; exit 1; }
tail -2 $O/${T}_pytest_gpu.txt
timeout -k 10 400 python tools/ab_interleaved.py $L $L tinyraytracerinrust_amd/build/librt_mi355x_r3.so --reps 20 --burst 10 --check --option - 6=1 - > $O/${T}_ab.txt 2>&1 || { tail -20 $O/${T}_ab.txt; exit 1; }
grep -v amdgpu.ids $O/${T}_ab.txt
timeout -k 10 400 python tools/inflight_probe.py $L --ns 8,4 --ks 1 --reps 3 --options 7=0 - 6=1,7=0 6=1 > $O/${T}_inflight.txt 2>&1 || { tail -20 $O/${T}_inflight.txt; exit 1; }
grep -v amdgpu.ids $O/${T}_inflight.txt
echo session done
