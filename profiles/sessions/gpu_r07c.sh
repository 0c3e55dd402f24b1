#!/bin/bash
# Round 5: tiles-per-wave probe first (short), then the whole GPU suite and the bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r07c}
timeout -k 10 300 python -u tools/tpw_probe.py > $O/${T}_tpw.txt 2>&1 || { tail -20 $O/${T}_tpw.txt; exit 1; }
cat $O/${T}_tpw.txt
TAG=$T CONFIGS=1 KT=${KT:-0} bash tools/gpu_r4.sh
