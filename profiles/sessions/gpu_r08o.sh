#!/bin/bash
# Round 5: XCD-aware tile order WITH plain (write-back) frame stores, against the product (cost-sorted
# order, streaming stores) and plain stores alone: does one XCD's L2 merge a 128-B line's four tile
# row segments when they are stored through the cache?  Time per frame (A/B) and WRITE_SIZE.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r08o}
P=tinyraytracerinrust_amd/librt_mi355x.so
X=tinyraytracerinrust_amd/build/librt_mi355x_xcdp.so
Q=tinyraytracerinrust_amd/build/librt_mi355x_plain.so
for C in globes4k globes1080d5 sphere1080d0; do
  timeout -k 10 300 python -u tools/ab_libs.py $P $X $Q --config $C >> $O/${T}_xcdp_ab.txt 2>&1 || { tail -20 $O/${T}_xcdp_ab.txt; exit 1; }
done
cat $O/${T}_xcdp_ab.txt
for L in base xcdp plain; do
  LP=$P; [ $L = xcdp ] && LP=$X; [ $L = plain ] && LP=$Q
  for PMC in FETCH_SIZE WRITE_SIZE; do
    RT_LIB_PATH=$LP timeout -s KILL 150 rocprofv3 --pmc $PMC --output-format csv -d $O/${T}_${L}_4k_pmc_$PMC -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra > /dev/null 2> $O/${T}_${L}_4k_$PMC.err || { echo "pmc $PMC failed"; tail $O/${T}_${L}_4k_$PMC.err; exit 1; }
    RT_LIB_PATH=$LP timeout -s KILL 240 rocprofv3 --pmc $PMC --output-format csv -d $O/${T}_${L}_anim_pmc_$PMC -o run -- python3 bench.py --config anim120 --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $O/${T}_${L}_anim_$PMC.err || { echo "anim pmc $PMC failed"; tail $O/${T}_${L}_anim_$PMC.err; exit 1; }
  done
  python3 tools/pmc_quick.py ${T}_${L}_4k_pmc_ rt_spec_rows_00
  python3 tools/pmc_quick.py ${T}_${L}_anim_pmc_ rt_spec_rows_00
done
echo session done
