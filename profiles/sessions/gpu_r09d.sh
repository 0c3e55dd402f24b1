#!/bin/bash
# Round 6, session r09d: pool slots holding the hit object instead of w (RT_POOL_OBJ_INDEX): the GPU
# suite at the new binary, then the anim120 sweep of per-lane LDS frames / pool slots (RT_SPEC_KL /
# RT_SPEC_KP, diagnostic library): bench value + FETCH / WRITE per variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r09d}
sha256sum tinyraytracerinrust_amd/librt_mi355x.so | cut -c1-16 > $O/${T}_so_sha16.txt
( while sleep 50; do date +%T >> $O/${T}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_pytest_gpu.txt 2>&1 || { tail -40 $O/${T}_pytest_gpu.txt; exit 1; }
  tail -2 $O/${T}_pytest_gpu.txt
fi
E=tinyraytracerinrust_amd/ab/librt_mi355x_env.so
for V in ${VARIANTS:-1:122 1:183 0:265 0:320 1:238}; do
  KL=${V%%:*}; KP=${V##*:}
  TT=${T}_anim_${KL}_${KP}
  RT_LIB_PATH=$E RT_SPEC_KL=$KL RT_SPEC_KP=$KP timeout -k 10 400 python bench.py --config anim120 --steps 3 --warmup 2 --no-cpu-baseline > $O/${TT}.json 2> $O/${TT}.err || { tail $O/${TT}.err; exit 1; }
  for PMC in FETCH_SIZE WRITE_SIZE; do
    RT_LIB_PATH=$E RT_SPEC_KL=$KL RT_SPEC_KP=$KP timeout -s KILL 240 rocprofv3 --pmc $PMC --output-format csv -d $O/${TT}_pmc_$PMC -o run -- python3 bench.py --config anim120 --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $O/${TT}_pmc_$PMC.err || { echo "anim pmc $PMC failed"; tail $O/${TT}_pmc_$PMC.err; exit 1; }
  done
  python3 -c "import json;d=json.load(open('$O/${TT}.json'));print('anim120 KL=$KL KP=$KP', d['value'], d['ms_per_step'], d.get('frame_check'))"
  python3 tools/pmc_quick.py ${TT}_pmc_ rt_spec_rows_00 | grep -v "over"
done
echo session done
