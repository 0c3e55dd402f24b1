#!/bin/bash
# Round-2 GPU session: GPU tests (incl. full-size parity), default bench, host CPU facts.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-r02a}
python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())" > $OUT/${TAG}_host.txt
cat /sys/fs/cgroup/cpu.max >> $OUT/${TAG}_host.txt 2>&1 || true
grep -m1 "model name" /proc/cpuinfo >> $OUT/${TAG}_host.txt || true
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/${TAG}_pytest_gpu.txt 2>&1 || { tail -40 $OUT/${TAG}_pytest_gpu.txt; exit 1; }
tail -3 $OUT/${TAG}_pytest_gpu.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err || { tail $OUT/${TAG}_bench.err; exit 1; }
cat $OUT/${TAG}_bench.json
echo done
