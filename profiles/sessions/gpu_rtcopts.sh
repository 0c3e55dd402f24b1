#!/bin/bash
# hipRTC / LLVM scheduling options for the specialised 4K megakernel (diag build, RT_SPEC_OPTS),
# one process per variant (the process cache keys programs by their text), base first and last.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r06k}
D=tinyraytracerinrust_amd/build/librt_mi355x_dbg.so
i=0
for V in "" "-mllvm -amdgpu-sched-strategy=max-ilp" "-mllvm -amdgpu-schedule-metric-bias=0" "-mllvm -misched-postra" "-mllvm -amdgpu-sched-strategy=max-memory-clause" "-mllvm -amdgpu-schedule-metric-bias=100" ""; do
  i=$((i+1))
  RT_SPEC_OPTS="$V" timeout -k 10 200 python -u tools/ab_interleaved.py $D --option 6=1 --reps 40 --burst 4 > $O/${T}_$i.txt 2>&1 || { echo "variant [$V] failed"; tail -5 $O/${T}_$i.txt; continue; }
  echo "[$V] $(grep median $O/${T}_$i.txt | cut -c1-60)"
done
