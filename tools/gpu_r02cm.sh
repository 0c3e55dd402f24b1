# Shared sphere terms in the reflection-only megakernel (RT_SHARE_MEGA, sm1) vs product, after the
# oriented boxes freed registers.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
B=tinyraytracerinrust_amd/build
P=tinyraytracerinrust_amd/librt_mi355x.so
L="$P $B/librt_mi355x_sm1.so"
timeout -k 10 300 python tools/ab_interleaved.py $L --reps 15 --burst 10 > $O/r02cm_ab.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab_interleaved.py $L --reps 15 --burst 10 --depth 0 >> $O/r02cm_ab.txt 2>&1 || exit 1
grep -v amdgpu $O/r02cm_ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 400 --timeout-method thread -m gpu 2>&1 | tail -1
