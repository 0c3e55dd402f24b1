# Refraction frames' pending-reflection state: first frame in LDS (product, KLR=1) vs pend bit
# mask only (KLR=0) vs HEAD (scratch arrays); parity subset.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
B=tinyraytracerinrust_amd/build
P=tinyraytracerinrust_amd/librt_mi355x.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -m gpu -k "spinning or edge or ray_debugger or record or points" > $O/r02bk_pytest.txt 2>&1 || { tail -30 $O/r02bk_pytest.txt; exit 1; }
tail -1 $O/r02bk_pytest.txt
for t in 0.1 0.6; do
timeout -k 10 300 python tools/ab_interleaved.py $B/librt_mi355x_head.so $B/librt_mi355x_klr0.so $P --reps 12 --burst 10 --size 1920x1080 --scene spinning_globes --time $t >> $O/r02bk_ab.txt 2>&1 || exit 1
done
grep -v amdgpu $O/r02bk_ab.txt
