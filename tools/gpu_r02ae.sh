set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
L=tinyraytracerinrust_amd
timeout -k 10 300 python tools/ab_interleaved.py $L/librt_mi355x.so $L/build/librt_mi355x_mega.so --reps 12 --burst 10 --size 1920x1080 --depth 5 > $O/r02ae_ab.txt 2>&1 || exit 1
cat $O/r02ae_ab.txt
timeout -k 10 300 python tools/inflight_probe.py $L/librt_mi355x.so > $O/r02ae_inflight_auto.txt 2>&1 || exit 1
RT_DEFERRED=0 timeout -k 10 300 python tools/inflight_probe.py $L/librt_mi355x.so > $O/r02ae_inflight_mega.txt 2>&1 || exit 1
paste $O/r02ae_inflight_auto.txt $O/r02ae_inflight_mega.txt | awk -F'\t' '{print substr($1,1,30), "|", substr($2,6,25)}'
