#!/bin/bash
# PMC passes of every BASELINE bench config's product kernel at the current binary (HBM traffic, executed
# FP64, issue counters), one rocprofv3 --pmc run per counter group (rocprofv3 does not split passes).
# Afterwards, in the build container: python3 tools/pmc_summary.py ${TAG}_<config> <config> <kernel>
# for each config (profiles/pmc_summary.json, which bench.py's roofline blocks read).
# usage (GPU box): TAG=r09z bash tools/gpu_pmc_all.sh [CONFIGS...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:?set TAG}
CONFIGS=${*:-globes4k sphere1080d0 globes1080d5 anim120}
for C in $CONFIGS; do
  sha256sum tinyraytracerinrust_amd/librt_mi355x.so | cut -c1-16 > $O/${T}_${C}_so_sha16.txt
  case $C in
    globes4k) ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-extra"; LIM=150 ;;
    anim120) ARGS="--config anim120 --steps 1 --warmup 0 --no-cpu-baseline"; LIM=240 ;;
    *) ARGS="--config $C --steps 5 --warmup 1 --no-cpu-baseline --no-extra"; LIM=150 ;;
  esac
  for PMC in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64" "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES" "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"; do
    N=$(echo $PMC | tr ' ' '_' | cut -c1-40)
    timeout -s KILL $LIM rocprofv3 --pmc $PMC --output-format csv -d $O/${T}_${C}_pmc_$N -o run -- python3 bench.py $ARGS > /dev/null 2> $O/${T}_${C}_pmc_$N.err || { echo "pmc $C $PMC failed"; tail $O/${T}_${C}_pmc_$N.err; exit 1; }
  done
  echo "pmc $C done"
done
