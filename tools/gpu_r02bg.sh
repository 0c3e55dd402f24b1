# N = 1: one frame at a time vs 4 frames in flight (own-queue streams), every globes config.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
: > $O/r02bg.txt
for C in globes4k sphere1080d0 globes1080d5; do for K in 1 4; do
  timeout -k 10 300 python bench.py --config $C --inflight $K --steps 40 --warmup 5 --no-cpu-baseline > $O/r02bg_${C}_k$K.json 2> $O/r02bg.err || { tail $O/r02bg.err; exit 1; }
  python -c "
import json
d=json.loads(open('$O/r02bg_${C}_k$K.json').read().strip().splitlines()[-1]); print('$C K=$K', d['value'], d['ms_per_step'], d['frame_check'])" >> $O/r02bg.txt
done; done
cat $O/r02bg.txt
