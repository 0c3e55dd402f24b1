# Parity of the shared-sphere refraction kernels (+ new edge scene), A/B on spinning_globes, and
# the anim120 / globes4k bench lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
B=tinyraytracerinrust_amd/build
P=tinyraytracerinrust_amd/librt_mi355x.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fastclamp.py tests/test_gpu_deferred.py tests/test_gpu_fullsize.py tests/test_gpu_antialias.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/r02an_pytest.txt 2>&1 || { tail -30 $O/r02an_pytest.txt; exit 1; }
tail -2 $O/r02an_pytest.txt
for t in 0.1 0.6; do
timeout -k 10 300 python tools/ab_interleaved.py $B/librt_mi355x_noshare.so $P --reps 12 --burst 10 --size 1920x1080 --scene spinning_globes --time $t >> $O/r02an_ab.txt 2>&1 || exit 1
done
cat $O/r02an_ab.txt
timeout -k 10 300 python bench.py --config anim120 --steps 5 --warmup 2 > $O/r02an_bench_anim120.json 2> $O/r02an_bench_anim.err || { tail $O/r02an_bench_anim.err; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/r02an_bench.json 2> $O/r02an_bench.err || { tail $O/r02an_bench.err; exit 1; }
python -c "
import json
for f in ['$O/r02an_bench_anim120.json','$O/r02an_bench.json']:
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'], d['roofline']['frac'])"
