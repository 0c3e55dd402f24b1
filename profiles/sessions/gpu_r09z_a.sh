#!/bin/bash
# Round 6 consolidation, part A: PMC passes of every bench config at the round's product binary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
( while sleep 50; do date +%T >> gpurun_out/r09z_heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
TAG=r09z bash tools/gpu_pmc_all.sh globes4k sphere1080d0 globes1080d5 anim120 || exit 1
echo session done
