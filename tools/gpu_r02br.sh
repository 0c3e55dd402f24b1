# Up to 16-way splits of the costliest tiles (split16) vs 8 (product): 1080p d5 frame, N=4/8 shares.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
B=tinyraytracerinrust_amd/build
P=tinyraytracerinrust_amd/librt_mi355x.so
timeout -k 10 300 python tools/ab_interleaved.py $P $B/librt_mi355x_split16.so --reps 12 --burst 10 --size 1920x1080 --depth 5 > $O/r02br.txt 2>&1 || exit 1
timeout -k 10 300 python tools/inflight_probe.py $P $B/librt_mi355x_split16.so --ns 4,8 --ks 1 --reps 2 >> $O/r02br.txt 2>&1 || exit 1
RT_SPLIT_K=1 timeout -k 10 300 python tools/inflight_probe.py $B/librt_mi355x_split16.so --ns 4 --ks 1 --reps 2 >> $O/r02br.txt 2>&1 || exit 1
grep -v amdgpu $O/r02br.txt
