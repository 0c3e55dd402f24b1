#!/bin/bash
# Round 5: completion-mark cost A/B, anim120 LDS-frame variants, bench lines at HEAD.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r07d}
P=tinyraytracerinrust_amd/librt_mi355x.so
NM=tinyraytracerinrust_amd/build/librt_mi355x_nomarks.so
for C in sphere1080d0 globes1080d5 globes4k; do
  timeout -k 10 300 python -u tools/ab_libs.py $P $NM --config $C >> $O/${T}_marks_ab.txt 2>&1 || { tail -20 $O/${T}_marks_ab.txt; exit 1; }
done
cat $O/${T}_marks_ab.txt
for KL in 3 4 5 6; do
  RT_LIB_PATH=tinyraytracerinrust_amd/build/librt_mi355x_kl.so RT_SPEC_KL=$KL timeout -k 10 300 python bench.py --config anim120 --steps 3 --warmup 2 --no-cpu-baseline > $O/${T}_anim_kl$KL.json 2> $O/${T}_anim_kl$KL.err || { tail $O/${T}_anim_kl$KL.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/${T}_anim_kl$KL.json'));print('KL $KL', d['value'], d['ms_per_step'], d['roofline']['kernel'][:200])"
done
for C in globes4k sphere1080d0; do
  timeout -k 10 300 python bench.py --config $C --steps 20 --warmup 5 --no-cpu-baseline > $O/${T}_bench_$C.json 2> $O/${T}_bench_$C.err || { tail $O/${T}_bench_$C.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/${T}_bench_$C.json'));print('$C', d['value'], d['ms_per_step'], d['inflight4']['ms_per_step'], d['kernel_code'][:220])"
done
echo session done
