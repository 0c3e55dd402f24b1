set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
L=tinyraytracerinrust_amd
timeout -k 10 120 python tools/ab_interleaved.py $L/librt_mi355x.so --reps 5 --burst 20 > $O/r02l_same_box.txt 2>&1 || exit 1
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> $O/r02l_same_box.txt 2>&1 || exit 1
timeout -k 10 120 python bench.py --steps 100 --warmup 5 --no-cpu-baseline >> $O/r02l_same_box.txt 2>&1 || exit 1
timeout -k 10 120 python tools/ab_interleaved.py $L/librt_mi355x.so --reps 5 --burst 20 >> $O/r02l_same_box.txt 2>&1 || exit 1
cat $O/r02l_same_box.txt | cut -c1-400
