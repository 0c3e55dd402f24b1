# Shadow rays over the likeliest occluders first (strav) vs draw order (RT_DRAW_ORDER_SHADOWS=1 at upload).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
P=tinyraytracerinrust_amd/librt_mi355x.so
for a in "" "--depth 0" "--size 1920x1080 --depth 5"; do
  timeout -k 10 300 python tools/ab_interleaved.py $P $P --upload-env RT_DRAW_ORDER_SHADOWS=1 - --reps 15 --burst 10 $a >> $O/r02cr_ab.txt 2>&1 || exit 1
done
grep -v amdgpu $O/r02cr_ab.txt
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 400 --timeout-method thread -m gpu > $O/r02cr_pytest.txt 2>&1 || { tail -30 $O/r02cr_pytest.txt; exit 1; }
tail -1 $O/r02cr_pytest.txt
