#!/bin/bash
# Diagnostic: bench.py's default command and clean process exit (round 4: SIGSEGV after the JSON line).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
for i in 1 2; do
  timeout -k 5 180 python -X faulthandler bench.py --steps 20 --warmup 5 > $O/by_$i.json 2> $O/by_$i.err
  echo "[run $i] rc=$?"; grep -v amdgpu.ids $O/by_$i.err | tail -25
done
