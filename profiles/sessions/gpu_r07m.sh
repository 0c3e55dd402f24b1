#!/bin/bash
# Round 5: PMC passes of the 1080p configs at HEAD, the counter list, and an A/B of the specialised
# calibration kernel (RT_OPT_SPECIALIZE 2: the tile order measured by the specialised kernel itself).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
P=tinyraytracerinrust_amd/librt_mi355x.so
timeout -s KILL 60 rocprofv3 -L > $O/r07m_counters.txt 2>&1 || echo "counter list failed"
for C in globes4k globes1080d5; do
  timeout -k 10 300 python -u tools/ab_libs.py $P $P --levels 1,2 --config $C >> $O/r07m_spec_cal_ab.txt 2>&1 || { tail -20 $O/r07m_spec_cal_ab.txt; exit 1; }
done
cat $O/r07m_spec_cal_ab.txt
TAG=r07m bash tools/gpu_pmc_configs.sh
