#!/bin/bash
# A/B timing of library variants and host-side switches (diagnostic).  Each argument is
# "LIB[:ENV=VAL]"; the 4K globes kernel is timed for each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for spec in "$@"; do
  lib=${spec%%:*}; envs=""; [ "$spec" != "$lib" ] && envs=${spec#*:}
  echo "== $lib $envs"
  env $envs RT_LIB_PATH=$lib timeout -k 10 120 python tools/quick_timing.py 2>&1 | grep -v amdgpu.ids || exit 1
done
