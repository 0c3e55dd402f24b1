#!/bin/bash
# Round 6, session r09q: f64 culling back in the generic kernels (f32 in the specialised programs and
# the wavefront candidate walks): fractal, and the generic 4K frame, against the consolidation binary z.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r09q}
A=tinyraytracerinrust_amd/ab
N=tinyraytracerinrust_amd/librt_mi355x.so
for L in $A/librt_mi355x_z.so $N $A/librt_mi355x_z.so $N; do
  RT_LIB_PATH=$L timeout -k 10 300 python -u tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1 7 2>&1 | grep -v amdgpu.ids | sed "s|\$| [$(basename $L)]|" >> $O/${T}_fractal.txt || exit 1
done
cat $O/${T}_fractal.txt
timeout -k 10 300 python -u tools/ab_libs.py $A/librt_mi355x_z.so $N --config globes4k --generic > $O/${T}_ab.txt 2>&1 || { tail -20 $O/${T}_ab.txt; exit 1; }
timeout -k 10 300 python -u tools/ab_libs.py $A/librt_mi355x_z.so $N --config globes4k >> $O/${T}_ab.txt 2>&1 || { tail -20 $O/${T}_ab.txt; exit 1; }
grep -v amdgpu.ids $O/${T}_ab.txt
echo session done
