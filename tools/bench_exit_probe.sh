#!/bin/bash
# Diagnostic: bench.py phases and clean process exit (round 4: aborts / SIGSEGV after the JSON line).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
for v in "--no-extra --no-cpu-baseline --specialize 0" "--no-extra --no-cpu-baseline" "--no-cpu-baseline"; do
  N=$(echo $v | tr -d ' -')
  timeout -k 5 120 python bench.py --steps 5 --warmup 2 --settle-ms 50 $v > $O/bx_$N.json 2> $O/bx_$N.err
  echo "[$v] rc=$?"; grep -v amdgpu.ids $O/bx_$N.err | tail -3
done
