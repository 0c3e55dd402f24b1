#!/bin/bash
# Round 5: scalar-unit activity of the 4K headline kernel (how much of the CU's one scalar unit the
# specialised program's constant materialisation and exec-mask control occupy).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r08n}
PMC="SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
N=salu
timeout -s KILL 120 rocprofv3 --pmc $PMC --output-format csv -d $O/${T}_pmc_$N -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra > /dev/null 2> $O/${T}_pmc_$N.err || { echo "pmc failed"; tail -3 $O/${T}_pmc_$N.err; exit 1; }
python3 tools/pmc_quick.py ${T}_pmc_ rt_spec_rows_00
echo session done
