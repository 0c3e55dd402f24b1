#!/bin/bash
# Round 6, session r10e: anim120 with 1-4 render streams at the final binary (the default is 2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
for S in 2 1 3 4 2 3; do
  timeout -k 10 300 python bench.py --config anim120 --streams $S --steps 3 --warmup 2 --no-cpu-baseline --no-extra > $O/r10e_anim_s$S.json 2> $O/r10e_anim_s$S.err || { tail $O/r10e_anim_s$S.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/r10e_anim_s$S.json'));print('streams $S', d['value'], d['ms_per_step'])" | tee -a $O/r10e_anim_streams.txt
done
