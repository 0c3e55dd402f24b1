#!/bin/bash
# Round 6, session r09u: printf of every f32 box decision where the fma slab form and the sub/mul form
# disagree (diagnostic library pdbg, RT_CULL_DEBUG), on the cull-edge mismatch's points.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
P="865.9443037974686,770.3456701834464 865.9443037974686,770.3456701834465"
RT_LIB_PATH=tinyraytracerinrust_amd/ab/librt_mi355x_pdbg.so timeout -k 10 120 python -u tools/points_check.py profiles/sessions/cubes_edges.scene 1920 1080 10 $P > $O/r09u_culldiff.txt 2>&1 || { tail -20 $O/r09u_culldiff.txt; exit 1; }
grep -v amdgpu.ids $O/r09u_culldiff.txt | head -40
