#!/bin/bash
# Round 4 tuning with the ROCm 7.2 hipRTC: specialised kernels' waves per SIMD (diag builds sw3 /
# sw5 vs 4), rank shares at N = 2..8 (specialised), anim120 over 1 / 2 / 8 streams.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r05x}
M=tinyraytracerinrust_amd/librt_mi355x.so
B=tinyraytracerinrust_amd/build
( while sleep 50; do date +%T >> $O/${T}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 400 python -u tools/ab_interleaved.py $M $B/librt_mi355x_sw3.so $B/librt_mi355x_sw5.so --option 6=1 6=1 6=1 --reps 30 --burst 4 --check > $O/${T}_ab_waves4k.txt 2>&1 || { tail -20 $O/${T}_ab_waves4k.txt; exit 1; }
grep median $O/${T}_ab_waves4k.txt
timeout -k 10 400 python -u tools/ab_interleaved.py $M $B/librt_mi355x_sw3.so $B/librt_mi355x_sw5.so --option 6=1 6=1 6=1 --size 1920x1080 --depth 5 --reps 30 --burst 4 --check > $O/${T}_ab_waves1080.txt 2>&1 || { tail -20 $O/${T}_ab_waves1080.txt; exit 1; }
grep median $O/${T}_ab_waves1080.txt
timeout -k 10 400 python -u tools/rank_share_probe.py $M $B/librt_mi355x_sw3.so $B/librt_mi355x_sw5.so --spec > $O/${T}_shares.txt 2>&1 || { tail -20 $O/${T}_shares.txt; exit 1; }
grep -v amdgpu.ids $O/${T}_shares.txt
for K in 1 2 8; do
  timeout -k 10 400 python bench.py --config anim120 --steps 3 --warmup 1 --streams $K --no-cpu-baseline > $O/${T}_anim_s$K.json 2> $O/${T}_anim_s$K.err || { tail $O/${T}_anim_s$K.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/${T}_anim_s$K.json'));print('anim streams $K', d['value'], d['ms_per_step'])"
done
echo session done
