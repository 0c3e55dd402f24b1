# RCCL stream priority (high vs normal) on the RCCL path at world 1 with 4 frames in flight.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
: > $O/r02bw.txt
for r in 1 2; do for pr in high normal; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2955$r bench.py --force-collective --inflight 4 --steps 40 --warmup 5 --no-cpu-baseline --rccl-priority $pr > $O/r02bw_$pr$r.json 2> $O/r02bw.err || { tail $O/r02bw.err; exit 1; }
  python -c "
import json
d=json.loads(open('$O/r02bw_$pr$r.json').read().strip().splitlines()[-1]); print('$pr', d['value'], d['ms_per_step'], d['distributed']['frame_check'])" >> $O/r02bw.txt
done; done
cat $O/r02bw.txt
