# AA pass: trace kernel with one-wave groups + LDS frames (product) vs HEAD; AA parity tests.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_antialias.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/r02bm_pytest.txt 2>&1 || { tail -30 $O/r02bm_pytest.txt; exit 1; }
tail -1 $O/r02bm_pytest.txt
for r in 1 2; do
RT_LIB_PATH=tinyraytracerinrust_amd/build/librt_mi355x_head.so timeout -k 10 200 python tools/aa_timing.py 2>&1 | grep -v amdgpu | sed 's/^/HEAD /' >> $O/r02bm_aa.txt || exit 1
timeout -k 10 200 python tools/aa_timing.py 2>&1 | grep -v amdgpu | sed 's/^/new  /' >> $O/r02bm_aa.txt || exit 1
done
cat $O/r02bm_aa.txt
