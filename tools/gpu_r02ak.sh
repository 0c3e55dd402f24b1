set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r02ak_pytest.txt 2>&1 || { tail -40 $O/r02ak_pytest.txt; exit 1; }
tail -2 $O/r02ak_pytest.txt
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29551 bench.py --gpus 1 --steps 20 --warmup 5 --force-collective --inflight 4 > $O/r02ak_bench_collective_rgb.json 2> $O/r02ak_bench_collective_rgb.err || { tail -20 $O/r02ak_bench_collective_rgb.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/r02ak_bench_collective_rgb.json')); print(d['value'], d['config']['collective'], d['distributed'])"
