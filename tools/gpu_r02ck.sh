# Calibration on a cold GPU vs after one warm-up launch (RT_CAL_LAUNCHES): the 1080p d5 config line
# and the A/B tool with the same library twice (the second context calibrates warm), 4K globes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
P=tinyraytracerinrust_amd/librt_mi355x.so
for n in 1 2 3; do
  echo "RT_CAL_LAUNCHES=$n"
  RT_CAL_LAUNCHES=$n timeout -k 10 120 python tools/ab_interleaved.py $P $P --reps 15 --burst 10 --size 1920x1080 --depth 5 2>&1 | grep -v amdgpu
  for i in 1 2 3; do
    RT_CAL_LAUNCHES=$n timeout -k 10 120 python bench.py --config globes1080d5 --steps 20 --warmup 2 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('  bench 1080p d5', d['ms_per_step'], d['roofline']['kernel_ms_mean'])"
    RT_CAL_LAUNCHES=$n timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('  bench 4K d10', d['ms_per_step'], d['roofline']['kernel_ms_mean'])"
  done
done
