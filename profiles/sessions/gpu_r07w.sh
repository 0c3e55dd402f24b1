#!/bin/bash
# Round 5: camera terms of integer pixels from per-column / per-row tables, single-band row fast path:
# the whole GPU suite, then A/B against the previous library on the BASELINE configs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r07w}
P=tinyraytracerinrust_amd/librt_mi355x.so
V=tinyraytracerinrust_amd/build/librt_mi355x_prev.so
( while sleep 50; do date +%T >> $O/${T}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_pytest_gpu.txt 2>&1 || { tail -40 $O/${T}_pytest_gpu.txt; exit 1; }
tail -2 $O/${T}_pytest_gpu.txt
for C in sphere1080d0 globes1080d5 globes4k; do
  timeout -k 10 300 python -u tools/ab_libs.py $V $P --config $C >> $O/${T}_ab.txt 2>&1 || { tail -20 $O/${T}_ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/${T}_ab.txt
echo session done
