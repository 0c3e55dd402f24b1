#!/bin/bash
# Round 6, session r09x: RtDevScene's compact-node pointers moved to its end (the specialised kernels'
# argument offsets as in z) against the previous build (p0) and z.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
A=tinyraytracerinrust_amd/ab
N=tinyraytracerinrust_amd/librt_mi355x.so
for C in globes4k globes1080d5 sphere1080d0; do
  timeout -k 10 600 python -u tools/ab_libs.py $N $A/librt_mi355x_p0.so $A/librt_mi355x_z.so --config $C >> $O/r09x_ab.txt 2>&1 || { tail -20 $O/r09x_ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/r09x_ab.txt
echo session done
