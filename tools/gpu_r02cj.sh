# Spread of the 1080p depth-5 config line across fresh processes (each calibrates its own tile
# order and split factors), library's choice vs the megakernel forced.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
for i in 1 2 3 4 5; do
  timeout -k 10 120 python bench.py --config globes1080d5 --steps 20 --warmup 2 --no-cpu-baseline > $O/r02cj_auto_$i.json 2>/dev/null || exit 1
  RT_DEFERRED=0 timeout -k 10 120 python bench.py --config globes1080d5 --steps 20 --warmup 2 --no-cpu-baseline > $O/r02cj_mega_$i.json 2>/dev/null || exit 1
done
python3 - <<'P'
import json
for k in ("auto", "mega"):
    for i in range(1, 6):
        d = json.load(open(f"gpurun_out/r02cj_{k}_{i}.json"))
        print(k, i, d["value"], d["ms_per_step"], d["roofline"]["kernel_ms_mean"], d["roofline"]["kernel_ms_min"])
P
