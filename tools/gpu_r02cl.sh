# Calibration over summed launches (RT_CAL_LAUNCHES 1 / 3 / 5): spread of the 1080p d5 config line
# over fresh processes, and the 4K headline.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
for n in 1 3 5; do
  echo "RT_CAL_LAUNCHES=$n"
  for i in 1 2 3 4 5 6; do
    RT_CAL_LAUNCHES=$n timeout -k 10 120 python bench.py --config globes1080d5 --steps 20 --warmup 2 --no-cpu-baseline --settle-ms 150 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('  bench 1080p d5', d['ms_per_step'], d['roofline']['kernel_ms_mean'])"
  done
  RT_CAL_LAUNCHES=$n timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('  bench 4K d10', d['ms_per_step'], d['roofline']['kernel_ms_mean'])"
done
