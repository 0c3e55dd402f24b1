#!/bin/bash
# The tail kernel: a rank's N = 8 / 4 share (K = 1) with RT_OPT_TAIL_TILES 0 / 64 / 128, generic and
# specialised, then a kernel trace (rocprofv3 --kernel-trace --stats) of the N = 8 share with 64 tiles.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; T=${TAG:-r05e}; mkdir -p $O
L=tinyraytracerinrust_amd/librt_mi355x.so
timeout -k 10 400 python tools/inflight_probe.py $L --ns 8,4 --ks 1 --reps 2 --options 7=0 7=64 7=128 6=1,7=0 6=1,7=64 6=1,7=128 > $O/${T}_tail_shares.txt 2>&1 || { tail -20 $O/${T}_tail_shares.txt; exit 1; }
grep -v amdgpu.ids $O/${T}_tail_shares.txt
timeout -k 10 400 python tools/ab_interleaved.py $L tinyraytracerinrust_amd/build/librt_mi355x_sw4.so --reps 20 --burst 10 --check --option 6=1 6=1 > $O/${T}_ab_w4.txt 2>&1 || { tail -20 $O/${T}_ab_w4.txt; exit 1; }
grep -v amdgpu.ids $O/${T}_ab_w4.txt
for opt in 7=64 6=1,7=64; do
  N=$(echo $opt | tr ',=' '__')
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_kt_$N -o run -- python3 tools/inflight_probe.py $L --ns 8 --ks 1 --reps 1 --frames 20 --options $opt > $O/${T}_kt_$N.txt 2>&1 || { tail $O/${T}_kt_$N.txt; exit 1; }
done
echo done
