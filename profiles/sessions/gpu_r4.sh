#!/bin/bash
# One GPU-box session (round 4).  Every GPU step has its own time limit and the chain stops at the
# first failure (no retries).  Knobs: TAG (file prefix), TESTS=0 skips pytest, PYTEST_ARGS, AB="lib..."
# interleaved A/B of library builds (AB_ARGS: extra ab_interleaved.py arguments), CONFIGS=1 adds every
# BASELINE config's bench line, KT=0 skips the rocprofv3 kernel trace, PMC=1 adds the PMC passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r05x}
sha256sum tinyraytracerinrust_amd/librt_mi355x.so | cut -c1-16 > $O/${T}_so_sha16.txt
( while sleep 50; do date +%T >> $O/${T}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $O/${T}_pytest_gpu.txt 2>&1 || { tail -40 $O/${T}_pytest_gpu.txt; exit 1; }
  tail -2 $O/${T}_pytest_gpu.txt
fi
if [ -n "${AB:-}" ]; then
  timeout -k 10 600 python tools/ab_interleaved.py $AB ${AB_ARGS:-} > $O/${T}_ab.txt 2>&1 || { tail -20 $O/${T}_ab.txt; exit 1; }
  cat $O/${T}_ab.txt
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/${T}_bench.json 2> $O/${T}_bench.err || { tail $O/${T}_bench.err; exit 1; }
  cat $O/${T}_bench.json
fi
if [ "${CONFIGS:-0}" = "1" ]; then
  for C in sphere1080d0 globes1080d5 anim120; do
    S=20; [ $C = anim120 ] && S=3
    timeout -k 10 300 python bench.py --config $C --steps $S --warmup 2 > $O/${T}_bench_$C.json 2> $O/${T}_bench_$C.err || { tail $O/${T}_bench_$C.err; exit 1; }
    cat $O/${T}_bench_$C.json
  done
fi
if [ "${PMC:-0}" = "1" ]; then
  for PMC in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64" "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES" "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"; do
    N=$(echo $PMC | tr ' ' '_' | cut -c1-40)
    timeout -s KILL 120 rocprofv3 --pmc $PMC --output-format csv -d $O/${T}_pmc_$N -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra ${PMC_ARGS:-} > /dev/null 2> $O/${T}_pmc_$N.err || { echo "pmc pass $PMC failed (see $O/${T}_pmc_$N.err)"; exit 1; }
  done
fi
# the kernel trace runs bench.py WITH its extra phase (own-queue streams), which is what crashed the
# profiler's teardown in round 3 (streams now destroyed before exit, raytracer.py HwStream)
if [ "${KT:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_kt -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/${T}_bench_kt.json 2> $O/${T}_kt.err || { tail $O/${T}_kt.err; exit 1; }
fi
echo session done
