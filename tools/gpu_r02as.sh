# Leaf box tests dropped where they cannot cull (or cost what the shared sphere terms cost), in
# scenes with a transparent object: parity, A/B against HEAD's flattening, anim120 line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
B=tinyraytracerinrust_amd/build
P=tinyraytracerinrust_amd/librt_mi355x.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -m gpu -k "spinning or edge or cost_ordered or dsl" > $O/r02as_pytest.txt 2>&1 || { tail -30 $O/r02as_pytest.txt; exit 1; }
tail -1 $O/r02as_pytest.txt
for t in 0.1 0.3 0.6; do
timeout -k 10 300 python tools/ab_interleaved.py $B/librt_mi355x_relax0.so $P --reps 12 --burst 10 --size 1920x1080 --scene spinning_globes --time $t >> $O/r02as_ab.txt 2>&1 || exit 1
done
cat $O/r02as_ab.txt
timeout -k 10 300 python bench.py --config anim120 --steps 5 --warmup 2 > $O/r02as_bench_anim120.json 2> $O/r02as_bench_anim.err || { tail $O/r02as_bench_anim.err; exit 1; }
python -c "
import json
d=json.loads(open('$O/r02as_bench_anim120.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
