set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
L=tinyraytracerinrust_amd
B=$L/build
timeout -k 10 300 python tools/ab_interleaved.py $L/librt_mi355x.so $B/librt_mi355x_w5.so $B/librt_mi355x_w6.so --reps 10 --burst 10 > $O/r02r_ab.txt 2>&1 || { tail $O/r02r_ab.txt; exit 1; }
timeout -k 10 300 python tools/ab_interleaved.py $L/librt_mi355x.so $B/librt_mi355x_w5.so $B/librt_mi355x_w6.so --reps 10 --burst 10 --size 3840x1080 >> $O/r02r_ab.txt 2>&1 || { tail $O/r02r_ab.txt; exit 1; }
cat $O/r02r_ab.txt
for V in w5 w6; do for C in FETCH_SIZE WRITE_SIZE; do
  RT_LIB_PATH=$B/librt_mi355x_$V.so timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/r02r_${V}_pmc_$C -o run -- python3 tools/render_loop.py 5 > /dev/null 2> $O/r02r_${V}.err || { tail $O/r02r_${V}.err; exit 1; }
done; done
echo done
