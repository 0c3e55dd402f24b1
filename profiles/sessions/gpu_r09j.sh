#!/bin/bash
# Round 6, session r09j: compact 32-byte hierarchy nodes (RtTravC) and f32 culling in the wavefront
# path (fractal regressed 5.39 -> 6.57 ms with the 96-byte RtTrav staged in LDS): the GPU suite, fractal
# timing of the consolidation binary (ab/librt_mi355x_z.so) and this one, and a 4K A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r09j}
sha256sum tinyraytracerinrust_amd/librt_mi355x.so | cut -c1-16 > $O/${T}_so_sha16.txt
( while sleep 50; do date +%T >> $O/${T}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_pytest_gpu.txt 2>&1 || { tail -40 $O/${T}_pytest_gpu.txt; exit 1; }
  tail -2 $O/${T}_pytest_gpu.txt
fi
for L in tinyraytracerinrust_amd/ab/librt_mi355x_z.so tinyraytracerinrust_amd/librt_mi355x.so tinyraytracerinrust_amd/ab/librt_mi355x_z.so tinyraytracerinrust_amd/librt_mi355x.so; do
  RT_LIB_PATH=$L timeout -k 10 300 python -u tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1 7 2>&1 | grep -v amdgpu.ids | sed "s|\$| [$(basename $L)]|" >> $O/${T}_fractal.txt || exit 1
done
cat $O/${T}_fractal.txt
timeout -k 10 300 python -u tools/ab_libs.py tinyraytracerinrust_amd/ab/librt_mi355x_z.so tinyraytracerinrust_amd/librt_mi355x.so --config globes4k > $O/${T}_ab.txt 2>&1 || { tail -20 $O/${T}_ab.txt; exit 1; }
grep -v amdgpu.ids $O/${T}_ab.txt
echo session done
