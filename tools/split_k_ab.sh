#!/bin/bash
# N = 8 / 4 single-frame share vs the split factor k (costly tiles: cost >= k * P * median -> P waves)
# and the split cap (P <= 8: etimes, P <= 16: etimes16).  Diagnostic builds only (RT_DIAG_SPLIT_K).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for L in etimes etimes16; do for k in 1.0 0.5 0.25 0.125; do for w in 8 4; do
  echo "== $L k=$k N=$w"
  RT_DIAG_SPLIT_K=$k timeout -k 10 120 python -u tools/entry_times_probe.py tinyraytracerinrust_amd/build/librt_mi355x_$L.so --world $w 2>&1 | grep -v amdgpu.ids | sed -n '1p;8,10p' || exit 1
done; done; done
