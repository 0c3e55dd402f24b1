#!/bin/bash
# Round 5: instruction-cache counters of the specialised row kernels (4K globes: 106 KB of code;
# the sphere: 14.5 KB), one SQC counter per pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r08h}
for C in globes4k sphere1080d0; do
  for PMC in "SQC_ICACHE_HITS SQ_WAVES SQ_IFETCH" "SQC_ICACHE_MISSES SQ_IFETCH_LEVEL" "SQC_ICACHE_MISSES_DUPLICATE SQ_WAIT_INST_ANY" "SQC_TC_INST_REQ SQ_INSTS_VALU"; do
    N=$(echo $PMC | tr ' ' '_' | cut -c1-40)
    timeout -s KILL 90 rocprofv3 --pmc $PMC --output-format csv -d $O/${T}_${C}_pmc_$N -o run -- python3 bench.py --config $C --steps 3 --warmup 1 --no-cpu-baseline --no-extra > /dev/null 2> $O/${T}_${C}_$N.err || { echo "pmc $C $PMC failed"; tail -3 $O/${T}_${C}_$N.err; exit 1; }
  done
  python3 tools/pmc_quick.py ${T}_${C}_pmc_ rt_spec_rows_00
done
echo session done
