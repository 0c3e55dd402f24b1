# Own-queue vs pool streams: N=1 K=4 without the collective, then with it (alternated).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
: > $O/r02be.txt
for r in 1 2; do for kind in hw pool; do
  X=""; [ $kind = pool ] && X="--pool-streams"
  timeout -k 10 300 python bench.py --inflight 4 --steps 40 --warmup 5 --no-cpu-baseline $X > $O/r02be_$kind$r.json 2> $O/r02be.err || { tail $O/r02be.err; exit 1; }
  python -c "
import json
d=json.loads(open('$O/r02be_$kind$r.json').read().strip().splitlines()[-1]); print('no collective', '$kind', d['value'], d['ms_per_step'])" >> $O/r02be.txt
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2954$r bench.py --force-collective --inflight 4 --steps 40 --warmup 5 --no-cpu-baseline $X > $O/r02be_c$kind$r.json 2> $O/r02be.err || { tail $O/r02be.err; exit 1; }
  python -c "
import json
d=json.loads(open('$O/r02be_c$kind$r.json').read().strip().splitlines()[-1]); print('collective', '$kind', d['value'], d['ms_per_step'])" >> $O/r02be.txt
done; done
cat $O/r02be.txt
