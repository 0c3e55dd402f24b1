# Constant hit filters (RtLeaf::filter_const) vs evaluated (RT_NO_CONST_FILTER=1 at upload).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
P=tinyraytracerinrust_amd/librt_mi355x.so
for a in "" "--depth 0" "--size 1920x1080 --scene spinning_globes --time 0.3"; do
  timeout -k 10 300 python tools/ab_interleaved.py $P $P --upload-env RT_NO_CONST_FILTER=1 - --reps 15 --burst 10 $a >> $O/r02co_ab.txt 2>&1 || exit 1
done
grep -v amdgpu $O/r02co_ab.txt
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 400 --timeout-method thread -m gpu > $O/r02co_pytest.txt 2>&1 || { tail -30 $O/r02co_pytest.txt; exit 1; }
tail -1 $O/r02co_pytest.txt
timeout -k 10 300 python bench.py --config anim120 --steps 3 --warmup 2 > $O/r02co_bench_anim120.json 2>/dev/null || exit 1; cut -c1-200 $O/r02co_bench_anim120.json
