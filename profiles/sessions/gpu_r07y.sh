#!/bin/bash
# Round 5 refresh at HEAD (camera-term tables): every config's bench line, PMC passes of all four
# configs' render kernels, the headline kernel trace; the sphere line also at 500 steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r07y}
TESTS=0 TAG=$T bash tools/gpu_final.sh || exit 1
TAG=$T bash tools/gpu_pmc_configs.sh || exit 1
timeout -k 10 300 python bench.py --config sphere1080d0 --steps 500 --warmup 20 > $O/${T}_bench_sphere1080d0_500.json 2> $O/${T}_b3.err || exit 1
python3 -c "import json;d=json.load(open('$O/${T}_bench_sphere1080d0_500.json'));print('sphere 500 steps', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_mean'])"
echo refresh done
