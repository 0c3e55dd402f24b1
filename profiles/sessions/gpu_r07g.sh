#!/bin/bash
# Round 5: frame pool sizes (anim120, 4K) against per-lane LDS frames; speed and HBM traffic.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r07g}
P=tinyraytracerinrust_amd/librt_mi355x.so
KLL=tinyraytracerinrust_amd/build/librt_mi355x_kl.so
for C in globes4k globes1080d5; do
  RT_SPEC_KL=2 timeout -k 10 300 python -u tools/ab_libs.py $P $KLL --config $C >> $O/${T}_pool_refl_ab.txt 2>&1 || { tail -20 $O/${T}_pool_refl_ab.txt; exit 1; }
done
cat $O/${T}_pool_refl_ab.txt
run_anim() {   # name, env...
  local N=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config anim120 --steps 10 --warmup 2 --no-cpu-baseline > $O/${T}_anim_$N.json 2> $O/${T}_anim_$N.err || { tail $O/${T}_anim_$N.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/${T}_anim_$N.json'));print('anim $N', d['value'], d['ms_per_step'], d['roofline']['kernel'][:170])"
}
run_anim pool186 RT_X=0 || exit 1
run_anim kp250 RT_LIB_PATH=$KLL RT_SPEC_KP=250 || exit 1
run_anim kp314 RT_LIB_PATH=$KLL RT_SPEC_KP=314 || exit 1
run_anim kp120 RT_LIB_PATH=$KLL RT_SPEC_KP=120 || exit 1
run_anim kl1 RT_LIB_PATH=$KLL RT_SPEC_KL=1 || exit 1
run_anim kl2 RT_LIB_PATH=$KLL RT_SPEC_KL=2 || exit 1
for V in "kp250 RT_SPEC_KP=250" "kp314 RT_SPEC_KP=314" "kl1 RT_SPEC_KL=1"; do
  set -- $V
  for PMC in FETCH_SIZE WRITE_SIZE; do
    env RT_LIB_PATH=$KLL $2 timeout -s KILL 240 rocprofv3 --pmc $PMC --output-format csv -d $O/${T}a_$1_$PMC -o run -- python3 bench.py --config anim120 --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $O/${T}a_$1_$PMC.err || { echo "pmc $1 $PMC failed"; tail $O/${T}a_$1_$PMC.err; exit 1; }
  done
done
echo session done
