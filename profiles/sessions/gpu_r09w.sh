#!/bin/bash
# Round 6, session r09w: the texel guard's rare path as a call in the generic kernels (noinline
# sphere_uv_cr) against the guard inlined (z) and no guard (gts); the specialised 4K frame; fractal.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
A=tinyraytracerinrust_amd/ab
N=tinyraytracerinrust_amd/librt_mi355x.so
timeout -k 10 600 python -u tools/ab_libs.py $N $A/librt_mi355x_z.so $A/librt_mi355x_gts.so --config globes4k --generic > $O/r09w_ab.txt 2>&1 || { tail -20 $O/r09w_ab.txt; exit 1; }
timeout -k 10 600 python -u tools/ab_libs.py $N $A/librt_mi355x_z.so --config globes4k >> $O/r09w_ab.txt 2>&1 || { tail -20 $O/r09w_ab.txt; exit 1; }
grep -v amdgpu.ids $O/r09w_ab.txt
for L in $A/librt_mi355x_z.so $N $A/librt_mi355x_gts.so $N; do
  RT_LIB_PATH=$L timeout -k 10 300 python -u tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1 7 2>&1 | grep -v amdgpu.ids | sed "s|\$| [$(basename $L)]|" >> $O/r09w_fractal.txt || exit 1
done
cat $O/r09w_fractal.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_texel_boundary.py tests/test_gpu_cull_edges.py tests/test_gpu_parity.py > $O/r09w_tests.txt 2>&1 || { tail -30 $O/r09w_tests.txt; exit 1; }
tail -2 $O/r09w_tests.txt
echo session done
