set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 --force-collective > $O/r02p_bench_collective.json 2> $O/r02p_bench_collective.err || { tail -20 $O/r02p_bench_collective.err; exit 1; }
cat $O/r02p_bench_collective.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 1 --steps 20 --warmup 5 --force-collective --layout contiguous --inflight 2 > $O/r02p_bench_collective_contig.json 2> $O/r02p_bench_collective_contig.err || { tail -20 $O/r02p_bench_collective_contig.err; exit 1; }
cat $O/r02p_bench_collective_contig.json
