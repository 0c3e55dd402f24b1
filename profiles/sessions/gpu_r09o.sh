#!/bin/bash
# Round 6, session r09o: compact 32-byte hierarchy nodes in the generic walks (RtTravC): the GPU suite,
# fractal (round-5 library, the consolidation binary z, HEAD), and interleaved A/B z vs HEAD.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r09o}
sha256sum tinyraytracerinrust_amd/librt_mi355x.so | cut -c1-16 > $O/${T}_so_sha16.txt
( while sleep 50; do date +%T >> $O/${T}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
A=tinyraytracerinrust_amd/ab
N=tinyraytracerinrust_amd/librt_mi355x.so
for L in $A/librt_mi355x_cff8ab5a.so $A/librt_mi355x_z.so $N $A/librt_mi355x_cff8ab5a.so $N; do
  RT_LIB_PATH=$L timeout -k 10 300 python -u tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p1 7 2>&1 | grep -v amdgpu.ids | sed "s|\$| [$(basename $L)]|" >> $O/${T}_fractal.txt || exit 1
done
cat $O/${T}_fractal.txt
for C in globes4k sphere1080d0 globes1080d5; do
  timeout -k 10 300 python -u tools/ab_libs.py $A/librt_mi355x_z.so $N --config $C >> $O/${T}_ab.txt 2>&1 || { tail -20 $O/${T}_ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/${T}_ab.txt
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_pytest_gpu.txt 2>&1 || { tail -40 $O/${T}_pytest_gpu.txt; exit 1; }
  tail -2 $O/${T}_pytest_gpu.txt
fi
echo session done
