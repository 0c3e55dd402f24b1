#!/bin/bash
# Round 4: lone-frame rank shares (K = 1) with the specialised programs: the library's choice with the
# specialised tail ratio (2.5) and without it (diag build tr1, ratio 1.0), forced megakernel, forced
# deferred; and the 1080p d5 frame.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r06d}
M=tinyraytracerinrust_amd/librt_mi355x.so
R1=tinyraytracerinrust_amd/build/librt_mi355x_tr1.so
for K in auto mega deferred; do
  timeout -k 10 300 python -u tools/inflight_probe.py $M --options 6=1 --ks 1 --kernel $K --reps 2 > $O/${T}_$K.txt 2>&1 || { tail -20 $O/${T}_$K.txt; exit 1; }
  grep "N=" $O/${T}_$K.txt
done
timeout -k 10 300 python -u tools/inflight_probe.py $R1 --options 6=1 --ks 1 --kernel auto --reps 2 > $O/${T}_tr1.txt 2>&1 || { tail -20 $O/${T}_tr1.txt; exit 1; }
grep "N=" $O/${T}_tr1.txt
timeout -k 10 300 python -u tools/ab_interleaved.py $M $R1 $M $M --option 6=1 6=1 6=1 6=1 --kernel auto auto mega deferred --size 1920x1080 --depth 5 --reps 30 --burst 4 --check > $O/${T}_k1080.txt 2>&1 || { tail -20 $O/${T}_k1080.txt; exit 1; }
grep median $O/${T}_k1080.txt
# the calibrations' tail ratios (diag build: RT_TILE_ORDER_DEBUG prints max / (sum / slots))
D=tinyraytracerinrust_amd/build/librt_mi355x_dbg.so
RT_TILE_ORDER_DEBUG=1 timeout -k 10 300 python -u tools/inflight_probe.py $D --options 6=1 --ks 1 --kernel auto --reps 1 > $O/${T}_ratios.txt 2>&1 || { tail -20 $O/${T}_ratios.txt; exit 1; }
RT_TILE_ORDER_DEBUG=1 timeout -k 10 300 python -u tools/ab_interleaved.py $D --option 6=1 --size 1920x1080 --depth 5 --reps 3 >> $O/${T}_ratios.txt 2>&1 || { tail -20 $O/${T}_ratios.txt; exit 1; }
grep -E "tile order|N=|median" $O/${T}_ratios.txt | cut -c1-220
