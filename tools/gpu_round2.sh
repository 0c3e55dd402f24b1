#!/bin/bash
# One GPU-box session (round 2): GPU tests, default bench line, rank-share / in-flight probe,
# rocprofv3 kernel trace + PMC passes of the bench command.  Every GPU step has its own time limit
# and the chain stops at the first failure (no retries).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
TAG=${TAG:-r02x}
L=tinyraytracerinrust_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${TAG}_pytest_gpu.txt 2>&1 || { tail -40 $O/${TAG}_pytest_gpu.txt; exit 1; }
tail -2 $O/${TAG}_pytest_gpu.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { tail $O/${TAG}_bench.err; exit 1; }
cat $O/${TAG}_bench.json
[ "${PROBES:-1}" = "1" ] && { timeout -k 10 300 python tools/inflight_probe.py $L/librt_mi355x.so > $O/${TAG}_inflight.txt 2>&1 || { tail $O/${TAG}_inflight.txt; exit 1; }; cat $O/${TAG}_inflight.txt; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_kt -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/${TAG}_bench_kt.json 2> $O/${TAG}_kt.err || { tail $O/${TAG}_kt.err; exit 1; }
[ "${PMC_PASSES:-1}" = "1" ] || { echo done; exit 0; }
for PMC in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64" "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES" "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY"; do
  N=$(echo $PMC | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 120 rocprofv3 --pmc $PMC --output-format csv -d $O/${TAG}_pmc_$N -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> $O/${TAG}_pmc_$N.err || { echo "pmc pass $PMC failed (see $O/${TAG}_pmc_$N.err)"; exit 1; }
done
echo done
