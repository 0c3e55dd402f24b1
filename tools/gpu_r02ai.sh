set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
B=tinyraytracerinrust_amd/build
for C in FETCH_SIZE WRITE_SIZE; do
  RT_LIB_PATH=$B/librt_mi355x_v6.so timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/r02ai_v6_pmc_$C -o run -- python3 tools/render_loop.py 5 > /dev/null 2> $O/r02ai.err || { tail $O/r02ai.err; exit 1; }
done
timeout -k 10 300 python tools/ab_interleaved.py tinyraytracerinrust_amd/librt_mi355x.so $B/librt_mi355x_v6.so --reps 12 --burst 10 > $O/r02ai_ab.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab_interleaved.py tinyraytracerinrust_amd/librt_mi355x.so $B/librt_mi355x_v6.so --reps 12 --burst 10 --size 1920x1080 --depth 0 --scene globes >> $O/r02ai_ab.txt 2>&1 || exit 1
cat $O/r02ai_ab.txt
