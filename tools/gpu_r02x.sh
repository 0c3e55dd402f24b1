set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
L=tinyraytracerinrust_amd/librt_mi355x.so
timeout -k 10 300 python tools/inflight_probe.py $L > $O/r02x_inflight_auto.txt 2>&1 || exit 1
RT_DEFERRED=0 timeout -k 10 300 python tools/inflight_probe.py $L > $O/r02x_inflight_mega.txt 2>&1 || exit 1
RT_DEFERRED=1 timeout -k 10 300 python tools/inflight_probe.py $L > $O/r02x_inflight_def.txt 2>&1 || exit 1
paste $O/r02x_inflight_auto.txt $O/r02x_inflight_mega.txt $O/r02x_inflight_def.txt | awk -F'\t' '{print substr($1,1,30), "|", substr($2,6,25), "|", substr($3,6,25)}'
