# Tile-count-dependent split factor: globes 1080p d5 frame, N = 4 / 8 rank shares (K = 1), and the
# deferred-kernel parity tests.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_deferred.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -m gpu -k "deferred or kernel_option or rank_bands or globes1080" > $O/r02bq_pytest.txt 2>&1 || { tail -30 $O/r02bq_pytest.txt; exit 1; }
tail -1 $O/r02bq_pytest.txt
timeout -k 10 300 python bench.py --config globes1080d5 --steps 40 --warmup 5 --no-cpu-baseline > $O/r02bq_1080.json 2> $O/r02bq.err || { tail $O/r02bq.err; exit 1; }
python -c "
import json
d=json.loads(open('$O/r02bq_1080.json').read().strip().splitlines()[-1]); print('globes1080d5', d['value'], d['ms_per_step'])"
timeout -k 10 200 python tools/inflight_probe.py tinyraytracerinrust_amd/librt_mi355x.so --ns 4,8 --ks 1 --reps 2 2>&1 | grep -v amdgpu
