#!/bin/bash
# LDS stack frames of the specialised megakernel (RT_SPEC_LDS_FRAMES diag builds kl3/kl4/kl5 vs the
# default 2): interleaved timing, then HBM FETCH/WRITE passes of each build's bench run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r05h}
B=tinyraytracerinrust_amd/build
( while sleep 50; do date +%T >> $O/${T}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u tools/ab_interleaved.py tinyraytracerinrust_amd/librt_mi355x.so $B/librt_mi355x_kl3.so $B/librt_mi355x_kl4.so $B/librt_mi355x_kl5.so --option 6=1 6=1 6=1 6=1 --reps 30 --burst 4 --check > $O/${T}_ab.txt 2>&1 || { tail -20 $O/${T}_ab.txt; exit 1; }
cat $O/${T}_ab.txt
for V in base kl4 kl5; do
  L=tinyraytracerinrust_amd/librt_mi355x.so; [ $V != base ] && L=$B/librt_mi355x_$V.so
  for PMC in FETCH_SIZE WRITE_SIZE; do
    RT_LIB_PATH=$L timeout -s KILL 180 rocprofv3 --pmc $PMC --output-format csv -d $O/${T}_${V}_pmc_$PMC -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra > /dev/null 2> $O/${T}_${V}_pmc_$PMC.err || { echo "pmc $V $PMC failed"; tail $O/${T}_${V}_pmc_$PMC.err; exit 1; }
  done
done
echo session done
