#!/bin/bash
# Round 6, session r09v: the generic 4K frame (the kernels before the specialised program loads) ran
# 0.463 ms in r09c and 1.56-1.61 ms since; diagnostic builds without each later exact shortcut.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
A=tinyraytracerinrust_amd/ab
timeout -k 10 600 python -u tools/ab_libs.py tinyraytracerinrust_amd/librt_mi355x.so $A/librt_mi355x_e5.so $A/librt_mi355x_gts.so $A/librt_mi355x_gun.so $A/librt_mi355x_gif.so $A/librt_mi355x_gss.so --config globes4k --generic > $O/r09v_generic_ab.txt 2>&1 || { tail -20 $O/r09v_generic_ab.txt; exit 1; }
grep -v amdgpu.ids $O/r09v_generic_ab.txt
