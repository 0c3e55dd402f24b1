set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
L=tinyraytracerinrust_amd
B=$L/build
timeout -k 10 300 python tools/ab_interleaved.py $L/librt_mi355x.so $B/librt_mi355x_w5.so $B/librt_mi355x_w6.so $B/librt_mi355x_w8.so --reps 10 --burst 10 > $O/r02o_waves_sustained.txt 2>&1 || { tail $O/r02o_waves_sustained.txt; exit 1; }
cat $O/r02o_waves_sustained.txt
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/r02o_clock -o run -- python3 tools/render_loop.py 60 > /dev/null 2> $O/r02o_clock.err || { tail $O/r02o_clock.err; exit 1; }
ls $O/r02o_clock
