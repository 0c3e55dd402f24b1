set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
L=tinyraytracerinrust_amd
B=$L/build
timeout -k 10 300 python tools/ab_interleaved.py $L/librt_mi355x.so $B/librt_mi355x_dw5.so $B/librt_mi355x_dw6.so $B/librt_mi355x_dw8.so --reps 10 --burst 10 --size 1920x1080 --depth 5 > $O/r02s_ab.txt 2>&1 || { tail $O/r02s_ab.txt; exit 1; }
timeout -k 10 300 python tools/ab_interleaved.py $L/librt_mi355x.so $B/librt_mi355x_rw5.so $B/librt_mi355x_rw3.so --reps 10 --burst 10 --size 1920x1080 --scene spinning_globes --time 0.25 >> $O/r02s_ab.txt 2>&1 || { tail $O/r02s_ab.txt; exit 1; }
cat $O/r02s_ab.txt
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/r02s_prod4k_pmc_$C -o run -- python3 tools/render_loop.py 5 > /dev/null 2> $O/r02s_p.err || { tail $O/r02s_p.err; exit 1; }
done
echo done
