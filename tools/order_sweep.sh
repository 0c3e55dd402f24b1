#!/bin/bash
# Tile-order run-length sweep (diagnostic): kernel times of the quick_timing cases and spinning_globes
# for RT_ORDER_RUN in the given list, plus the row-major dispatch (RT_TILE_ORDER=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
echo "== row-major (RT_TILE_ORDER=0)"
RT_TILE_ORDER=0 timeout -k 10 120 python tools/quick_timing.py 2>&1 | grep -v amdgpu.ids || exit 1
RT_TILE_ORDER=0 timeout -k 10 120 python tools/ab_interleaved.py tinyraytracerinrust_amd/librt_mi355x.so --reps 20 --scene spinning_globes --size 1920x1080 2>&1 | grep -v amdgpu.ids || exit 1
for r in "$@"; do
  echo "== RT_ORDER_RUN=$r"
  RT_ORDER_RUN=$r timeout -k 10 120 python tools/quick_timing.py 2>&1 | grep -v amdgpu.ids || exit 1
  RT_ORDER_RUN=$r timeout -k 10 120 python tools/ab_interleaved.py tinyraytracerinrust_amd/librt_mi355x.so --reps 20 --scene spinning_globes --size 1920x1080 2>&1 | grep -v amdgpu.ids || exit 1
done
