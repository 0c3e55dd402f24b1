set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
L=tinyraytracerinrust_amd
timeout -k 10 200 python tools/tile_stats_probe.py $L/build/librt_mi355x_stats.so > $O/r02d_tile_stats.txt 2>&1 || { tail $O/r02d_tile_stats.txt; exit 1; }
timeout -k 10 200 python tools/tile_stats_probe.py $L/build/librt_mi355x_stats.so --world 8 >> $O/r02d_tile_stats.txt 2>&1 || { tail $O/r02d_tile_stats.txt; exit 1; }
cat $O/r02d_tile_stats.txt
timeout -k 10 300 python tools/inflight_probe.py $L/build/librt_mi355x_mega.so $L/librt_mi355x.so > $O/r02d_inflight.txt 2>&1 || { tail $O/r02d_inflight.txt; exit 1; }
cat $O/r02d_inflight.txt
