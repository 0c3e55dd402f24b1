#!/bin/bash
# Time the 4K globes kernel for each library variant given on the command line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for lib in "$@"; do
  echo "== $lib"
  RT_LIB_PATH=$lib timeout -k 10 120 python tools/quick_timing.py 2>&1 | grep -v amdgpu.ids || exit 1
done
