set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
L=tinyraytracerinrust_amd
B=$L/build
timeout -k 10 300 python tools/ab_interleaved.py $L/librt_mi355x.so $B/librt_mi355x_lg2.so $B/librt_mi355x_lg4.so $B/librt_mi355x_w5.so --reps 10 --burst 10 > $O/r02q_ab.txt 2>&1 || { tail $O/r02q_ab.txt; exit 1; }
cat $O/r02q_ab.txt
for V in lg2 w5; do
  RT_LIB_PATH=$B/librt_mi355x_$V.so timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE --output-format csv -d $O/r02q_${V}_pmc_fw -o run -- python3 tools/render_loop.py 5 > /dev/null 2> $O/r02q_${V}.err || { tail $O/r02q_${V}.err; exit 1; }
done
RT_LIB_PATH=$L/librt_mi355x.so timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE --output-format csv -d $O/r02q_prod_pmc_fw -o run -- python3 tools/render_loop.py 5 > /dev/null 2> $O/r02q_prod.err || { tail $O/r02q_prod.err; exit 1; }
echo done
