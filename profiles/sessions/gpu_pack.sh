#!/bin/bash
# Packed pixel stores (store_pixels) vs per-lane stores (diag build np, RT_PACK_STORES=0): the store
# tests, interleaved timing, the write calibration (background-only 4K frame) and the bench WRITE /
# FETCH passes of both builds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r05k}
B=tinyraytracerinrust_amd/build
M=tinyraytracerinrust_amd/librt_mi355x.so
( while sleep 50; do date +%T >> $O/${T}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_stores.py tests/test_gpu_tail.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/${T}_pytest.txt 2>&1 || { tail -40 $O/${T}_pytest.txt; exit 1; }
tail -2 $O/${T}_pytest.txt
L="$M $B/librt_mi355x_np.so"
timeout -k 10 300 python -u tools/ab_interleaved.py $L $L --option 6=1 6=1 - - --reps 30 --burst 4 --check > $O/${T}_ab4k.txt 2>&1 || { tail -20 $O/${T}_ab4k.txt; exit 1; }
cat $O/${T}_ab4k.txt
timeout -k 10 300 python -u tools/ab_interleaved.py $L --option 6=1 6=1 --size 1920x1080 --depth 5 --reps 30 --burst 4 --check > $O/${T}_ab1080.txt 2>&1 || { tail -20 $O/${T}_ab1080.txt; exit 1; }
cat $O/${T}_ab1080.txt
timeout -k 10 300 python -u tools/ab_interleaved.py $L --size 1920x1080 --depth 0 --scene sphere --reps 40 --burst 8 --check > $O/${T}_absphere.txt 2>&1 || { tail -20 $O/${T}_absphere.txt; exit 1; }
cat $O/${T}_absphere.txt
for V in base np; do
  L=$M; [ $V != base ] && L=$B/librt_mi355x_$V.so
  for PMC in WRITE_SIZE FETCH_SIZE; do
    RT_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --pmc $PMC --output-format csv -d $O/${T}_${V}_wcal_$PMC -o run -- python3 tools/write_calib.py > $O/${T}_${V}_wcal_$PMC.log 2>&1 || { echo "wcal $V $PMC failed"; tail $O/${T}_${V}_wcal_$PMC.log; exit 1; }
    RT_LIB_PATH=$L timeout -s KILL 180 rocprofv3 --pmc $PMC --output-format csv -d $O/${T}_${V}_pmc_$PMC -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra > /dev/null 2> $O/${T}_${V}_pmc_$PMC.err || { echo "pmc $V $PMC failed"; tail $O/${T}_${V}_pmc_$PMC.err; exit 1; }
  done
done
echo session done
