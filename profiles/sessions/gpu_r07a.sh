#!/bin/bash
# Round 5, first session: the inflight-phase investigation and a PC-sampling
# attempt on the specialised 4K megakernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=r07a
timeout -k 10 240 python -u tools/inflight_bench_probe.py --rounds 3 > $O/${T}_inflight_4k.txt 2>&1 || { tail -20 $O/${T}_inflight_4k.txt; exit 1; }
cat $O/${T}_inflight_4k.txt | tail -14
timeout -k 10 240 python -u tools/inflight_bench_probe.py --rounds 3 --config sphere1080d0 --frames 200 > $O/${T}_inflight_sphere.txt 2>&1 || { tail -20 $O/${T}_inflight_sphere.txt; exit 1; }
tail -14 $O/${T}_inflight_sphere.txt
timeout -s KILL 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 -d $O/${T}_pcs -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-extra --settle-ms 0 > $O/${T}_pcs_bench.json 2> $O/${T}_pcs.err || { echo "pc sampling failed rc=$?"; tail -20 $O/${T}_pcs.err; }
ls -laR $O/${T}_pcs | head -30
echo session done
