#!/bin/bash
# Nontemporal frame stores (diag build nt, RT_NT_STORES, generic kernels) vs plain stores: counted
# HBM writes of the background-only frame and of 4K globes, and interleaved timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r06h}
M=tinyraytracerinrust_amd/librt_mi355x.so
N=tinyraytracerinrust_amd/build/librt_mi355x_nt.so
timeout -k 10 300 python -u tools/ab_interleaved.py $M $N --reps 30 --burst 4 --check > $O/${T}_ab.txt 2>&1 || { tail -20 $O/${T}_ab.txt; exit 1; }
grep median $O/${T}_ab.txt
for V in base nt; do
  L=$M; [ $V = nt ] && L=$N
  RT_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${T}_${V}_wcal -o run -- python3 tools/write_calib.py > $O/${T}_${V}_wcal.log 2>&1 || { tail $O/${T}_${V}_wcal.log; exit 1; }
  RT_LIB_PATH=$L timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${T}_${V}_pmc -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra --specialize 0 > /dev/null 2> $O/${T}_${V}_pmc.err || { tail $O/${T}_${V}_pmc.err; exit 1; }
done
echo done
