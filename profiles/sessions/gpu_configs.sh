# Bench lines for every BASELINE config on one MI355X (N = 1), each under its own time limit.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
TAG=${TAG:-r02m}
for C in globes4k sphere1080d0 globes1080d5 anim120; do
  S=20; [ $C = anim120 ] && S=3
  timeout -k 10 300 python bench.py --config $C --steps $S --warmup 2 > $O/${TAG}_bench_$C.json 2> $O/${TAG}_bench_$C.err || { tail $O/${TAG}_bench_$C.err; exit 1; }
  cat $O/${TAG}_bench_$C.json
done
