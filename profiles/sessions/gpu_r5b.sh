#!/bin/bash
# Round-4 session b: GPU tests (incl. the specialised and tail kernels), the spec A/B at 4K, and the
# N = 8 / 4 single-frame shares with the tail kernel and specialisation on / off.  The specialised
# kernels' tests compile with hipRTC for up to a minute each: a heartbeat file under gpurun_out/
# marks the session alive, pytest's own --timeout bounds every test.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; T=${TAG:-r05c}; mkdir -p $O
L=tinyraytracerinrust_amd/librt_mi355x.so
( while sleep 50; do date +%T >> $O/${T}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $O/${T}_pytest_gpu.txt 2>&1 || { tail -40 $O/${T}_pytest_gpu.txt; exit 1; }
  tail -2 $O/${T}_pytest_gpu.txt
fi
timeout -k 10 400 python tools/ab_interleaved.py $L $L tinyraytracerinrust_amd/build/librt_mi355x_r3.so --reps 20 --burst 10 --check --option - 6=1 - > $O/${T}_ab.txt 2>&1 || { tail -20 $O/${T}_ab.txt; exit 1; }
grep -v amdgpu.ids $O/${T}_ab.txt
timeout -k 10 400 python tools/inflight_probe.py $L --ns 8,4 --ks 1 --reps 3 --options 7=0 - 6=1,7=0 6=1 > $O/${T}_inflight.txt 2>&1 || { tail -20 $O/${T}_inflight.txt; exit 1; }
grep -v amdgpu.ids $O/${T}_inflight.txt
echo session done
