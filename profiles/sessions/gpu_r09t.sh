#!/bin/bash
# Round 6, session r09t: the cull-edge mismatch with the sub/mul slab form (pfs) and with RtTrav nodes in the
# generic f32 walks (ptc) instead of the compact RtTravC.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r09t}
A=tinyraytracerinrust_amd/ab
P="865.9443037974686,770.3456701834461 865.9443037974686,770.3456701834464 865.9443037974686,770.3456701834465 865.9443037974686,770.3456701834468"
for L in tinyraytracerinrust_amd/librt_mi355x.so $A/librt_mi355x_pfs.so $A/librt_mi355x_ptc.so; do
  RT_LIB_PATH=$L timeout -k 10 120 python -u tools/points_check.py profiles/sessions/cubes_edges.scene 1920 1080 10 $P 2>&1 | grep -v amdgpu.ids >> $O/${T}_points.txt
  rc=$?; [ $rc -ge 124 ] && { echo "points_check rc $rc on $L"; exit 1; }
  RT_LIB_PATH=$L timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -s tests/test_gpu_cull_edges.py > $O/${T}_edges_$(basename $L .so).txt 2>&1
  rc=$?; [ $rc -ge 2 ] && { echo "pytest rc $rc on $L"; tail -20 $O/${T}_edges_$(basename $L .so).txt; exit 1; }
  echo "== $L" >> $O/${T}_summary.txt
  grep -E "points at|passed|failed|AssertionError: \[" $O/${T}_edges_$(basename $L .so).txt | cut -c1-400 >> $O/${T}_summary.txt
done
cat $O/${T}_points.txt $O/${T}_summary.txt
echo session done
