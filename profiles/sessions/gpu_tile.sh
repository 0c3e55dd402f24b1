#!/bin/bash
# Tile shape of the row kernels (RT_TILE_W diag builds t16 = 16x4, t32 = 32x2 vs the default 8x8):
# interleaved timing (specialised and generic, 4K d10 and 1080p d5, frames checked equal), then the
# HBM WRITE/FETCH passes of each build's bench run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r05j}
B=tinyraytracerinrust_amd/build
M=tinyraytracerinrust_amd/librt_mi355x.so
( while sleep 50; do date +%T >> $O/${T}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
L="$M $B/librt_mi355x_t16.so $B/librt_mi355x_t32.so"
timeout -k 10 300 python -u tools/ab_interleaved.py $L $L --option 6=1 6=1 6=1 - - - --reps 30 --burst 4 --check > $O/${T}_ab4k.txt 2>&1 || { tail -20 $O/${T}_ab4k.txt; exit 1; }
cat $O/${T}_ab4k.txt
timeout -k 10 300 python -u tools/ab_interleaved.py $L --option 6=1 6=1 6=1 --size 1920x1080 --depth 5 --reps 30 --burst 4 --check > $O/${T}_ab1080.txt 2>&1 || { tail -20 $O/${T}_ab1080.txt; exit 1; }
cat $O/${T}_ab1080.txt
timeout -k 10 300 python -u tools/ab_interleaved.py $L --size 1920x1080 --depth 0 --scene sphere --reps 30 --burst 4 --check > $O/${T}_absphere.txt 2>&1 || { tail -20 $O/${T}_absphere.txt; exit 1; }
cat $O/${T}_absphere.txt
for V in base t16 t32; do
  L=$M; [ $V != base ] && L=$B/librt_mi355x_$V.so
  for PMC in WRITE_SIZE FETCH_SIZE; do
    RT_LIB_PATH=$L timeout -s KILL 180 rocprofv3 --pmc $PMC --output-format csv -d $O/${T}_${V}_pmc_$PMC -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra > /dev/null 2> $O/${T}_${V}_pmc_$PMC.err || { echo "pmc $V $PMC failed"; tail $O/${T}_${V}_pmc_$PMC.err; exit 1; }
  done
done
echo session done
