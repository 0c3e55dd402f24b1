# RCCL path at world 1 (force-collective, K = 4): own-queue streams vs torch pool streams, alternated.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
: > $O/r02bd.txt
for r in 1 2; do for kind in hw pool; do
  X=""; [ $kind = pool ] && X="--pool-streams"
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2953$r bench.py --force-collective --inflight 4 --steps 40 --warmup 5 --no-cpu-baseline $X > $O/r02bd_$kind$r.json 2> $O/r02bd.err || { tail $O/r02bd.err; exit 1; }
  python -c "
import json
d=json.loads(open('$O/r02bd_$kind$r.json').read().strip().splitlines()[-1]); print('$kind', d['value'], d['ms_per_step'])" >> $O/r02bd.txt
done; done
cat $O/r02bd.txt
