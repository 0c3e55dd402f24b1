# Persistent megakernel (one wave per slot, work counter) vs one workgroup per tile: HEAD, the
# loop-structured kernel without persistence (product), persistent (pers).  Parity of pers.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
B=tinyraytracerinrust_amd/build
P=tinyraytracerinrust_amd/librt_mi355x.so
RT_LIB_PATH=$B/librt_mi355x_pers.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread -m gpu -k "not antialias" > $O/r02bx_pytest.txt 2>&1 || { tail -30 $O/r02bx_pytest.txt; exit 1; }
tail -1 $O/r02bx_pytest.txt
timeout -k 10 300 python tools/ab_interleaved.py $B/librt_mi355x_head.so $P $B/librt_mi355x_pers.so --reps 12 --burst 10 > $O/r02bx_ab.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab_interleaved.py $B/librt_mi355x_head.so $P $B/librt_mi355x_pers.so --reps 12 --burst 10 --size 1920x1080 --depth 0 >> $O/r02bx_ab.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab_interleaved.py $B/librt_mi355x_head.so $P $B/librt_mi355x_pers.so --reps 12 --burst 10 --size 1920x1080 --scene spinning_globes --time 0.3 >> $O/r02bx_ab.txt 2>&1 || exit 1
grep -v amdgpu $O/r02bx_ab.txt
