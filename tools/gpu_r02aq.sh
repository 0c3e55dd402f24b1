# Lane refill in the refraction kernel: parity (pool 2 = product; pool 4 through the env), then
# A/B of pools 1 / 2 / 4 on spinning_globes frames and the anim120 bench line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
B=tinyraytracerinrust_amd/build
P=tinyraytracerinrust_amd/librt_mi355x.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/r02aq_pytest.txt 2>&1 || { tail -30 $O/r02aq_pytest.txt; exit 1; }
tail -1 $O/r02aq_pytest.txt
RT_REFILL_POOL=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "spinning or shared or edge or cost_ordered or bands" > $O/r02aq_pytest4.txt 2>&1 || { tail -30 $O/r02aq_pytest4.txt; exit 1; }
tail -1 $O/r02aq_pytest4.txt
for t in 0.1 0.6; do
timeout -k 10 300 python tools/ab_interleaved.py $B/librt_mi355x_pool1.so $P $B/librt_mi355x_pool4.so --reps 12 --burst 10 --size 1920x1080 --scene spinning_globes --time $t >> $O/r02aq_ab.txt 2>&1 || exit 1
done
cat $O/r02aq_ab.txt
timeout -k 10 300 python bench.py --config anim120 --steps 5 --warmup 2 > $O/r02aq_bench_anim120.json 2> $O/r02aq_bench_anim.err || { tail $O/r02aq_bench_anim.err; exit 1; }
python -c "
import json
d=json.loads(open('$O/r02aq_bench_anim120.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
