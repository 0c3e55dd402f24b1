set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
L=tinyraytracerinrust_amd
B=$L/build
timeout -k 10 300 python tools/ab_interleaved.py $L/librt_mi355x.so $B/librt_mi355x_v4.so $B/librt_mi355x_v6.so $B/librt_mi355x_v7.so $B/librt_mi355x_v5l3.so --reps 10 --burst 10 > $O/r02ah_ab.txt 2>&1 || exit 1
cat $O/r02ah_ab.txt
