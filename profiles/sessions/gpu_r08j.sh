#!/bin/bash
# Round 5: chain-mode family programs at 7 waves/SIMD (RT_SPEC_WAVES_CHAIN=7) with smaller wave pools
# (so the LDS holds 7 one-wave workgroups per SIMD) against the product's 6 waves / 122 slots: anim120.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r08j}
B=tinyraytracerinrust_amd/build
run_anim() {   # name, env...
  local N=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config anim120 --steps 5 --warmup 2 --no-cpu-baseline > $O/${T}_anim_$N.json 2> $O/${T}_anim_$N.err || { tail $O/${T}_anim_$N.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/${T}_anim_$N.json'));print('anim $N', d['value'], d['ms_per_step'], d['kernel_code'] if 'kernel_code' in d else '', d['roofline']['kernel'][90:200])" | tee -a $O/${T}_anim.txt
}
for R in 1 2; do
  run_anim base RT_LIB_PATH=$B/librt_mi355x_denv.so || exit 1
  run_anim w7kp100 RT_LIB_PATH=$B/librt_mi355x_w7.so RT_SPEC_KP=100 || exit 1
  run_anim w7kp110 RT_LIB_PATH=$B/librt_mi355x_w7.so RT_SPEC_KP=110 || exit 1
  run_anim w6kp100 RT_LIB_PATH=$B/librt_mi355x_denv.so RT_SPEC_KP=100 || exit 1
done
echo session done
