# Bench lines with own-queue streams: N=1 default, force-collective K=4 (RCCL path at world 1),
# anim120; GPU tests.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/r02bb_bench.json 2> $O/r02bb_bench.err || { tail $O/r02bb_bench.err; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --force-collective --inflight 4 --steps 40 --warmup 5 --no-cpu-baseline > $O/r02bb_bench_collective.json 2> $O/r02bb_collective.err || { tail $O/r02bb_collective.err; exit 1; }
timeout -k 10 300 python bench.py --config anim120 --steps 3 --warmup 2 --no-cpu-baseline > $O/r02bb_bench_anim120.json 2> $O/r02bb_anim.err || { tail $O/r02bb_anim.err; exit 1; }
for f in r02bb_bench r02bb_bench_collective r02bb_bench_anim120; do python -c "
import json
d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d.get('frame_check') or d.get('distributed', {}).get('frame_check'))"; done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r02bb_pytest.txt 2>&1 || { tail -30 $O/r02bb_pytest.txt; exit 1; }
tail -1 $O/r02bb_pytest.txt
