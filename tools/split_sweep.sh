# Split-factor sweep for tail-bound launches (deferred kernel + split tiles): globes 1080p d5
# frame (BASELINE config 3, one frame at a time) and the N = 4 / 8 rank shares at K = 1.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
: > $O/r02bp.txt
for k in ${KS:-1.5 2 3}; do
  RT_SPLIT_K=$k timeout -k 10 300 python bench.py --config globes1080d5 --steps 40 --warmup 5 --no-cpu-baseline > $O/r02bp_$k.json 2> $O/r02bp.err || { tail $O/r02bp.err; exit 1; }
  python -c "
import json
d=json.loads(open('$O/r02bp_$k.json').read().strip().splitlines()[-1]); print('split_k $k globes1080d5', d['value'], d['ms_per_step'])" >> $O/r02bp.txt
  RT_SPLIT_K=$k timeout -k 10 200 python tools/inflight_probe.py tinyraytracerinrust_amd/librt_mi355x.so --ns 4,8 --ks 1 --reps 2 2>&1 | grep -v amdgpu | sed "s/^/split_k $k /" >> $O/r02bp.txt || exit 1
done
cat $O/r02bp.txt
