#!/bin/bash
# One GPU-box session: tests, bench, rocprofv3 kernel trace + PMC passes.  Every GPU step has
# its own time limit and the chain stops at the first failure (no retries).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-r01}
STEPS=${STEPS:-40}
run() { echo "== $*" >&2; "$@"; }
run timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/${TAG}_pytest_gpu.txt 2>&1 || { tail -30 $OUT/${TAG}_pytest_gpu.txt; exit 1; }
tail -3 $OUT/${TAG}_pytest_gpu.txt
run timeout -k 10 300 python bench.py --steps $STEPS --warmup 10 > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err || { cat $OUT/${TAG}_bench.err | tail; exit 1; }
cat $OUT/${TAG}_bench.json
run timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 5 --force-collective > $OUT/${TAG}_bench_collective.json 2> $OUT/${TAG}_bench_collective.err || { tail -20 $OUT/${TAG}_bench_collective.err; exit 1; }
cat $OUT/${TAG}_bench_collective.json
run timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_kt -o run -- python3 bench.py --steps $STEPS --warmup 10 --no-cpu-baseline > $OUT/${TAG}_bench_kt.json 2> $OUT/${TAG}_kt.err || { tail $OUT/${TAG}_kt.err; exit 1; }
[ "${PMC_PASSES:-1}" = "1" ] || { echo done; exit 0; }
run timeout -k 10 120 rocprofv3 -L > $OUT/${TAG}_counters.txt 2>&1 || true
for PMC in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64" "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES" "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY" "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64"; do
  N=$(echo $PMC | tr ' ' '_' | cut -c1-40)
  # a failed or timed-out pass ends the session: nothing more runs on the GPU after it
  run timeout -k 10 300 rocprofv3 --pmc $PMC --output-format csv -d $OUT/${TAG}_pmc_$N -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/${TAG}_pmc_$N.err || { echo "pmc pass $PMC failed (see $OUT/${TAG}_pmc_$N.err)"; exit 1; }
done
echo done
