#!/bin/bash
# Round 6, session r09i: the shadow walks' share of the 4K kernel (ablation library nosh: every shadow
# ray unoccluded, wrong pixels, timing only) and the product kernel's VALU / SALU per wave at this binary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r09i}
A=tinyraytracerinrust_amd/ab
N=tinyraytracerinrust_amd/librt_mi355x.so
timeout -k 10 300 python -u tools/ab_libs.py $N $A/librt_mi355x_nosh.so --config globes4k --no-check > $O/${T}_ab.txt 2>&1 || { tail -20 $O/${T}_ab.txt; exit 1; }
grep -v amdgpu.ids $O/${T}_ab.txt
for L in $N $A/librt_mi355x_nosh.so; do
  B=$(basename $L .so)
  RT_LIB_PATH=$L timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_BRANCH --output-format csv -d $O/${T}_${B}_pmc -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra > /dev/null 2> $O/${T}_${B}_pmc.err || { echo "pmc failed"; tail $O/${T}_${B}_pmc.err; exit 1; }
  python3 tools/pmc_quick.py ${T}_${B}_pmc rt_spec_rows_00
done
echo session done
