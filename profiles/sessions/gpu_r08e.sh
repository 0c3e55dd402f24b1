#!/bin/bash
# Round 5: the 1080p config lines at bench.py's default step counts (r08d's were overwritten by 20-step
# runs of the PMC script), and the sphere at 500 steps; same binary as r08d.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r08e}
sha256sum tinyraytracerinrust_amd/librt_mi355x.so | cut -c1-16 > $O/${T}_so_sha16.txt
for C in sphere1080d0 globes1080d5; do
  timeout -k 10 300 python bench.py --config $C > $O/${T}_bench_$C.json 2> $O/${T}_bench_$C.err || { tail $O/${T}_bench_$C.err; exit 1; }
done
timeout -k 10 300 python bench.py --config sphere1080d0 --steps 500 --warmup 20 > $O/${T}_bench_sphere1080d0_500.json 2> $O/${T}_b3.err || exit 1
for f in $O/${T}_bench*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', d['value'], d['ms_per_step'], d['steps'], d['roofline'].get('executed_fp64',{}).get('pmc_matches_binary'))"; done
echo session done
