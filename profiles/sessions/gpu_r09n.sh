#!/bin/bash
# Round 6, session r09n: instruction counts of the fractal frame's wf_trace_kernel, f64 culling (c64) vs
# f32 culling (HEAD): more work or slower work.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r09n}
A=tinyraytracerinrust_amd/ab
for L in $A/librt_mi355x_c64.so tinyraytracerinrust_amd/librt_mi355x.so; do
  B=$(basename $L .so)
  RT_LIB_PATH=$L timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_MUL_F64 --output-format csv -d $O/${T}_${B}_pmc -o run -- python3 tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1 2 > $O/${T}_${B}.txt 2>&1 || { tail $O/${T}_${B}.txt; exit 1; }
  python3 tools/pmc_quick.py ${T}_${B}_pmc wf_trace_kernel
done
echo session done
