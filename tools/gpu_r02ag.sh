set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r02ag_aa_kt -o run -- python3 tools/aa_timing.py > /dev/null 2>&1 || exit 1
cut -d, -f1-4 $O/r02ag_aa_kt/run_kernel_stats.csv | cut -c1-160
