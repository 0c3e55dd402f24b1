#!/bin/bash
# Verdict r2 item 3: scene tables staged in LDS (diagnostic build RT_DIAG_LDS_SCENE: 4 waves per
# workgroup share one LDS copy) against the product's scalar (SMEM) loads, 4K globes d10: interleaved
# kernel times with a bit-equality check, then one PMC pass per library (waits, VALU, waves).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r03q}
A=tinyraytracerinrust_amd/librt_mi355x.so
B=tinyraytracerinrust_amd/build/librt_mi355x_ldsscene.so
timeout -k 10 300 python -u tools/ab_interleaved.py $A $B --reps 30 --check > $O/${T}_lds_scene_ab.txt 2>&1 || { cat $O/${T}_lds_scene_ab.txt; exit 1; }
cat $O/${T}_lds_scene_ab.txt
for L in $A $B; do
  N=$(basename $L .so)
  RT_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SMEM --output-format csv -d $O/${T}_${N}_pmc_waits -o run -- python3 bench.py --steps 3 --warmup 1 --settle-ms 0 --no-cpu-baseline --no-extra > /dev/null 2> $O/${T}_${N}_pmc.err || { echo "pmc failed for $N"; tail $O/${T}_${N}_pmc.err; exit 1; }
done
python3 tools/pmc_ab.py $T
