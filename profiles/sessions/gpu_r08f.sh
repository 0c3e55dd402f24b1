#!/bin/bash
# Round 5: dynamic instruction classes of the 4K headline kernel (verdict item 4: attribute the
# non-FP64 instructions): two PMC passes of the SQ instruction-class counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r08f}
sha256sum tinyraytracerinrust_amd/librt_mi355x.so | cut -c1-16 > $O/${T}_so_sha16.txt
for PMC in "SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32" "SQ_WAVES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_FMA_F64"; do
  N=$(echo $PMC | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 150 rocprofv3 --pmc $PMC --output-format csv -d $O/${T}_pmc_$N -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra > /dev/null 2> $O/${T}_pmc_$N.err || { echo "pmc $PMC failed"; tail $O/${T}_pmc_$N.err; exit 1; }
done
python3 tools/pmc_quick.py ${T}_pmc_ rt_spec_rows_00
echo session done
