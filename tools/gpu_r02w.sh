set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
TAG=r02w bash tools/gpu_configs.sh > /dev/null || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/r02w_anim_pmc_$C -o run -- python3 bench.py --config anim120 --steps 1 --warmup 0 --settle-ms 0 --no-cpu-baseline > /dev/null 2> $O/r02w_anim.err || { tail $O/r02w_anim.err; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/r02w_g1080_pmc_$C -o run -- python3 bench.py --config globes1080d5 --steps 5 --warmup 0 --settle-ms 0 --no-cpu-baseline > /dev/null 2> $O/r02w_g.err || { tail $O/r02w_g.err; exit 1; }
done
echo done
