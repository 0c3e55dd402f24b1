#!/bin/bash
# Round 5: the wave frame pool -- GPU suite, bench lines, anim120 against the per-lane LDS frames, traffic.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r07f}
KLL=tinyraytracerinrust_amd/build/librt_mi355x_kl.so
( while sleep 50; do date +%T >> $O/${T}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_pytest_gpu.txt 2>&1 || { tail -40 $O/${T}_pytest_gpu.txt; exit 1; }
tail -2 $O/${T}_pytest_gpu.txt
for C in globes4k sphere1080d0 globes1080d5; do
  timeout -k 10 300 python bench.py --config $C --steps 20 --warmup 5 --no-cpu-baseline > $O/${T}_bench_$C.json 2> $O/${T}_bench_$C.err || { tail $O/${T}_bench_$C.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/${T}_bench_$C.json'));print('$C', d['value'], d['ms_per_step'], d['inflight4']['ms_per_step'], d['kernel_code'][:220])"
done
timeout -k 10 300 python bench.py --config anim120 --steps 10 --warmup 2 --no-cpu-baseline > $O/${T}_bench_anim120.json 2> $O/${T}_bench_anim120.err || { tail $O/${T}_bench_anim120.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/${T}_bench_anim120.json'));print('anim pool', d['value'], d['ms_per_step'], d['roofline']['kernel'][:200])"
for KL in 1 5; do
  RT_LIB_PATH=$KLL RT_SPEC_KL=$KL timeout -k 10 300 python bench.py --config anim120 --steps 10 --warmup 2 --no-cpu-baseline > $O/${T}_anim_kl$KL.json 2> $O/${T}_anim_kl$KL.err || { tail $O/${T}_anim_kl$KL.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/${T}_anim_kl$KL.json'));print('anim KL $KL', d['value'], d['ms_per_step'])"
done
for PMC in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $PMC --output-format csv -d $O/${T}a_pmc_$PMC -o run -- python3 bench.py --config anim120 --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $O/${T}a_pmc_$PMC.err || { echo "pmc $PMC failed"; tail $O/${T}a_pmc_$PMC.err; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc $PMC --output-format csv -d $O/${T}_pmc_$PMC -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra > /dev/null 2> $O/${T}_pmc_$PMC.err || { echo "pmc $PMC failed"; tail $O/${T}_pmc_$PMC.err; exit 1; }
done
echo session done
