#!/bin/bash
# Round 6, session r10c: kernel trace of the sphere bench (1 000 steps): the primary-ray kernel's own
# duration and the gaps between back-to-back launches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r10c_kt -o run -- python3 bench.py --config sphere1080d0 --no-cpu-baseline --no-extra > $O/r10c_bench_kt.json 2> $O/r10c_kt.err || { tail $O/r10c_kt.err; exit 1; }
head -4 $O/r10c_kt/run_kernel_stats.csv
