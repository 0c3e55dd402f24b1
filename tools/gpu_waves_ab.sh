set -o pipefail
export TMPDIR=/tmp
B=tinyraytracerinrust_amd/build
P=tinyraytracerinrust_amd/librt_mi355x.so
timeout -k 10 300 python tools/ab_interleaved.py $P $B/librt_mi355x_w4.so $B/librt_mi355x_w6.so --reps 12 --burst 10 2>&1 | grep -v amdgpu
timeout -k 10 300 python tools/ab_interleaved.py $P $B/librt_mi355x_w4.so $B/librt_mi355x_w6.so --reps 12 --burst 10 --depth 0 2>&1 | grep -v amdgpu
timeout -k 10 300 python tools/ab_interleaved.py $P $B/librt_mi355x_d5.so --reps 12 --burst 10 --size 1920x1080 --depth 5 2>&1 | grep -v amdgpu
