#!/bin/bash
# The tail kernel at issue priority 3: N = 8 / 4 shares (K = 1), generic and specialised; kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; T=${TAG:-r05f}; mkdir -p $O
L=tinyraytracerinrust_amd/librt_mi355x.so
timeout -k 10 400 python tools/inflight_probe.py $L --ns 8,4 --ks 1 --reps 2 --options 7=0 7=32 7=64 6=1,7=0 6=1,7=32 6=1,7=64 > $O/${T}_tail_shares.txt 2>&1 || { tail -20 $O/${T}_tail_shares.txt; exit 1; }
grep -v amdgpu.ids $O/${T}_tail_shares.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_kt -o run -- python3 tools/inflight_probe.py $L --ns 8 --ks 1 --reps 1 --frames 20 --options 6=1,7=64 > $O/${T}_kt.txt 2>&1 || { tail $O/${T}_kt.txt; exit 1; }
echo done
