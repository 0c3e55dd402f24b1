#!/bin/bash
# Round 6, session r10a: the GUI-shaped host (scene rebuilt and uploaded every frame at 480x360); tile orders kept across same-structure uploads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_gui_rebuild.py > $O/r10a_gui_rebuild.txt 2>&1 || { tail -40 $O/r10a_gui_rebuild.txt; exit 1; }
grep -E "rebuil|passed|failed" $O/r10a_gui_rebuild.txt
