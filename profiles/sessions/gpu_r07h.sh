#!/bin/bash
# Round 5: per-lane frames + wave pool (hybrid) against per-lane frames only and pool only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r07h}
P=tinyraytracerinrust_amd/librt_mi355x.so
KLL=tinyraytracerinrust_amd/build/librt_mi355x_kl.so
for C in globes4k globes1080d5; do
  RT_SPEC_KP=0 timeout -k 10 300 python -u tools/ab_libs.py $P $KLL --config $C >> $O/${T}_hybrid_refl_ab.txt 2>&1 || { tail -20 $O/${T}_hybrid_refl_ab.txt; exit 1; }
done
cat $O/${T}_hybrid_refl_ab.txt
run_anim() {   # name, env...
  local N=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config anim120 --steps 10 --warmup 2 --no-cpu-baseline > $O/${T}_anim_$N.json 2> $O/${T}_anim_$N.err || { tail $O/${T}_anim_$N.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/${T}_anim_$N.json'));print('anim $N', d['value'], d['ms_per_step'], d['roofline']['kernel'][:170])"
}
run_anim hybrid RT_X=0 || exit 1
run_anim kl1only RT_LIB_PATH=$KLL RT_SPEC_KL=1 RT_SPEC_KP=0 || exit 1
run_anim pool186 RT_LIB_PATH=$KLL RT_SPEC_KL=0 RT_SPEC_KP=186 || exit 1
run_anim hybrid2 RT_X=0 || exit 1
for PMC in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $PMC --output-format csv -d $O/${T}a_pmc_$PMC -o run -- python3 bench.py --config anim120 --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $O/${T}a_pmc_$PMC.err || { echo "pmc $PMC failed"; tail $O/${T}a_pmc_$PMC.err; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc $PMC --output-format csv -d $O/${T}_pmc_$PMC -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra > /dev/null 2> $O/${T}_pmc_$PMC.err || { echo "pmc $PMC failed"; tail $O/${T}_pmc_$PMC.err; exit 1; }
done
echo session done
