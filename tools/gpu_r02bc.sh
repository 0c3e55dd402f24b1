# Stream kinds for overlapping renders: CU-mask (own queue), plain hipStreamCreate, torch pool;
# 4 or 16 hardware queues.  A rank's N=8 / N=1 share with K = 4 frames in flight.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
P="python tools/inflight_probe.py tinyraytracerinrust_amd/librt_mi355x.so --ns 8,1 --ks 4 --reps 4 --measures 2"
{ echo "## hw (CU mask)"; timeout -k 10 200 $P --streams hw; } > $O/r02bc.txt 2>&1 || exit 1
{ echo "## plain hipStreamCreate"; RT_STREAM_PLAIN=1 timeout -k 10 200 $P --streams hw; } >> $O/r02bc.txt 2>&1 || exit 1
{ echo "## plain hipStreamCreate, GPU_MAX_HW_QUEUES=16"; RT_STREAM_PLAIN=1 GPU_MAX_HW_QUEUES=16 timeout -k 10 200 $P --streams hw; } >> $O/r02bc.txt 2>&1 || exit 1
{ echo "## torch pool, GPU_MAX_HW_QUEUES=16"; GPU_MAX_HW_QUEUES=16 timeout -k 10 200 $P --streams pool; } >> $O/r02bc.txt 2>&1 || exit 1
{ echo "## torch pool"; timeout -k 10 200 $P --streams pool; } >> $O/r02bc.txt 2>&1 || exit 1
grep -v amdgpu $O/r02bc.txt
