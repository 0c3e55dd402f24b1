set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
L=tinyraytracerinrust_amd
timeout -k 10 300 python tools/ab_interleaved.py $L/librt_mi355x.so $L/build/librt_mi355x_fc.so --reps 12 --burst 10 > $O/r02ab.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab_interleaved.py $L/librt_mi355x.so $L/build/librt_mi355x_fc.so --reps 12 --burst 10 --size 1920x1080 --scene spinning_globes --time 0.25 >> $O/r02ab.txt 2>&1 || exit 1
cat $O/r02ab.txt
