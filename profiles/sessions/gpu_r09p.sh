#!/bin/bash
# Round 6, session r09p: wf_trace_kernel on fractal, f64 (c64) vs f32 culling: wave-cycles, waits, issue,
# instruction-cache misses.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r09p}
A=tinyraytracerinrust_amd/ab
for L in $A/librt_mi355x_c64.so tinyraytracerinrust_amd/librt_mi355x.so; do
  B=$(basename $L .so)
  for PMC in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INST_CYCLES_SALU" "SQC_ICACHE_MISSES" "SQC_ICACHE_HITS" "SQC_DCACHE_MISSES" "SQC_DCACHE_HITS"; do
    N=$(echo $PMC | cut -d' ' -f1-2 | tr ' ' '_')
    RT_LIB_PATH=$L timeout -s KILL 200 rocprofv3 --pmc $PMC --output-format csv -d $O/${T}_${B}_pmc_$N -o run -- python3 tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1 2 > $O/${T}_${B}_$N.txt 2>&1 || { tail $O/${T}_${B}_$N.txt; exit 1; }
  done
  python3 tools/pmc_quick.py ${T}_${B}_pmc wf_trace_kernel
done
echo session done
