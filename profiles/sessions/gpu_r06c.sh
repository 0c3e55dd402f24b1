#!/bin/bash
# Round 4: kernel choice with the specialised programs (megakernel vs deferred at 1080p d5 / 4K d10)
# and frames in flight with specialisation (rank shares at N = 1..8, K = 1..4).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r06c}
M=tinyraytracerinrust_amd/librt_mi355x.so
( while sleep 50; do date +%T >> $O/${T}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 300 python -u tools/ab_interleaved.py $M $M $M --option 6=1 6=1 6=1 --kernel auto mega deferred --size 1920x1080 --depth 5 --reps 30 --burst 4 --check > $O/${T}_k1080.txt 2>&1 || { tail -20 $O/${T}_k1080.txt; exit 1; }
grep median $O/${T}_k1080.txt
timeout -k 10 300 python -u tools/ab_interleaved.py $M $M $M --option 6=1 6=1 6=1 --kernel auto mega deferred --reps 30 --burst 4 --check > $O/${T}_k4k.txt 2>&1 || { tail -20 $O/${T}_k4k.txt; exit 1; }
grep median $O/${T}_k4k.txt
timeout -k 10 400 python -u tools/inflight_probe.py $M --options 6=1 > $O/${T}_inflight.txt 2>&1 || { tail -20 $O/${T}_inflight.txt; exit 1; }
grep -v amdgpu.ids $O/${T}_inflight.txt | tail -25
echo session done
