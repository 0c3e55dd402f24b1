set -o pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_deferred.py tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread > $O/coop_tests.txt 2>&1 || { tail -30 $O/coop_tests.txt; exit 1; }
tail -1 $O/coop_tests.txt
timeout -k 10 300 python -u tools/inflight_probe.py tinyraytracerinrust_amd/librt_mi355x.so --ns 4,8 --ks 1 --reps 3 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python bench.py --config globes1080d5 --steps 20 --warmup 2 --no-cpu-baseline --no-extra 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('globes1080d5', d['value'], d['ms_per_step'])" || exit 1
