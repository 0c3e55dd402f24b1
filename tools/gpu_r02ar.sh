# Refill pool vs streams on anim120, and the tile-cost distribution of a spinning_globes frame.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
RT_TILE_ORDER_DEBUG=1 timeout -k 10 120 python tools/ab_interleaved.py tinyraytracerinrust_amd/librt_mi355x.so --reps 2 --size 1920x1080 --scene spinning_globes --time 0.3 > $O/r02ar_costs.txt 2>&1 || exit 1
RT_TILE_ORDER_DEBUG=1 timeout -k 10 120 python tools/ab_interleaved.py tinyraytracerinrust_amd/librt_mi355x.so --reps 2 --size 3840x2160 --scene globes >> $O/r02ar_costs.txt 2>&1 || exit 1
cat $O/r02ar_costs.txt
for P in 1 2 4; do for S in 2 4 8; do
RT_REFILL_POOL=$P timeout -k 10 300 python bench.py --config anim120 --steps 5 --warmup 2 --streams $S --no-cpu-baseline > $O/r02ar_anim_p${P}_s${S}.json 2> $O/r02ar_anim.err || { tail $O/r02ar_anim.err; exit 1; }
python -c "
import json
d=json.loads(open('$O/r02ar_anim_p${P}_s${S}.json').read().strip().splitlines()[-1]); print('pool $P streams $S', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_mean'])"
done; done
