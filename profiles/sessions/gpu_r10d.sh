#!/bin/bash
# Round 6, session r10d: the culling edge test over five scenes (silhouettes and shadow edges).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_cull_edges.py > gpurun_out/r10d_cull_edges.txt 2>&1; rc=$?
grep -E "points at|passed|failed|Error" gpurun_out/r10d_cull_edges.txt | cut -c1-300
exit $rc
