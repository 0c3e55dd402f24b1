#!/bin/bash
# PMC passes (HBM traffic, executed FP64, issue counters) of the globes1080d5 and sphere1080d0 bench
# configs at HEAD, for tools/pmc_summary.py (their bench lines' roofline blocks read them).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r06l}
for C in globes1080d5 sphere1080d0; do
  sha256sum tinyraytracerinrust_amd/librt_mi355x.so | cut -c1-16 > $O/${T}_${C}_so_sha16.txt
  for PMC in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64" "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES" "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"; do
    N=$(echo $PMC | tr ' ' '_' | cut -c1-40)
    timeout -s KILL 150 rocprofv3 --pmc $PMC --output-format csv -d $O/${T}_${C}_pmc_$N -o run -- python3 bench.py --config $C --steps 5 --warmup 1 --no-cpu-baseline --no-extra > /dev/null 2> $O/${T}_${C}_pmc_$N.err || { echo "pmc $C $PMC failed"; tail $O/${T}_${C}_pmc_$N.err; exit 1; }
  done
done
# (the config bench lines are gpu_final.sh's, at bench.py's default step counts; lines written here
# under the same names overwrote them in session r08d)
echo done
