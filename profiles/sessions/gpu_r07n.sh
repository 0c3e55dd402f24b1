#!/bin/bash
# Round 5: XCD-aware tile order (a 128-B line's tiles on one XCD, back to back) against the cost-sorted
# order: time per frame (A/B libraries) and the frame's HBM writes (WRITE_SIZE / FETCH_SIZE).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r07n}
P=tinyraytracerinrust_amd/librt_mi355x.so
X=tinyraytracerinrust_amd/build/librt_mi355x_xcd.so
for C in globes4k globes1080d5 sphere1080d0; do
  timeout -k 10 300 python -u tools/ab_libs.py $P $X --config $C >> $O/${T}_xcd_ab.txt 2>&1 || { tail -20 $O/${T}_xcd_ab.txt; exit 1; }
done
cat $O/${T}_xcd_ab.txt
run_anim() {   # name, env...
  local N=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config anim120 --steps 10 --warmup 2 --no-cpu-baseline > $O/${T}_anim_$N.json 2> $O/${T}_anim_$N.err || { tail $O/${T}_anim_$N.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/${T}_anim_$N.json'));print('anim $N', d['value'], d['ms_per_step'])"
}
run_anim base RT_X=0 || exit 1
run_anim xcd RT_LIB_PATH=$X || exit 1
run_anim base2 RT_X=0 || exit 1
run_anim xcd2 RT_LIB_PATH=$X || exit 1
for L in base xcd; do
  LP=$P; [ $L = xcd ] && LP=$X
  for PMC in FETCH_SIZE WRITE_SIZE; do
    RT_LIB_PATH=$LP timeout -s KILL 150 rocprofv3 --pmc $PMC --output-format csv -d $O/${T}_${L}_4k_pmc_$PMC -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra > /dev/null 2> $O/${T}_${L}_4k_$PMC.err || { echo "pmc $PMC failed"; tail $O/${T}_${L}_4k_$PMC.err; exit 1; }
    RT_LIB_PATH=$LP timeout -s KILL 240 rocprofv3 --pmc $PMC --output-format csv -d $O/${T}_${L}_anim_pmc_$PMC -o run -- python3 bench.py --config anim120 --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $O/${T}_${L}_anim_$PMC.err || { echo "anim pmc $PMC failed"; tail $O/${T}_${L}_anim_$PMC.err; exit 1; }
  done
  python3 tools/pmc_quick.py ${T}_${L}_4k_pmc_ rt_spec_rows_00
  python3 tools/pmc_quick.py ${T}_${L}_anim_pmc_ rt_spec_rows_00
done
echo session done
