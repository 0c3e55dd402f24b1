#!/bin/bash
# Round-end session at HEAD: the GPU test suite, every BASELINE config's bench line, the PMC passes of
# the headline and anim120 kernels (HBM traffic, executed FP64, issue counters -> pmc_summary.json via
# tools/pmc_summary.py afterwards), and a kernel trace of bench.py WITH its extra phase.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r06f}
sha256sum tinyraytracerinrust_amd/librt_mi355x.so | cut -c1-16 > $O/${T}_so_sha16.txt
cp $O/${T}_so_sha16.txt $O/${T}a_so_sha16.txt
( while sleep 50; do date +%T >> $O/${T}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_pytest_gpu.txt 2>&1 || { tail -40 $O/${T}_pytest_gpu.txt; exit 1; }
  tail -2 $O/${T}_pytest_gpu.txt
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/${T}_bench.json 2> $O/${T}_bench.err || { tail $O/${T}_bench.err; exit 1; }
# the config lines at bench.py's own defaults (50 steps, 10 warmup; anim120 3 animations of 120 frames)
for C in sphere1080d0 globes1080d5 anim120; do
  F=""; [ $C = anim120 ] && F="--steps 3 --warmup 2"
  timeout -k 10 400 python bench.py --config $C $F > $O/${T}_bench_$C.json 2> $O/${T}_bench_$C.err || { tail $O/${T}_bench_$C.err; exit 1; }
done
for PMC in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64" "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES" "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"; do
  N=$(echo $PMC | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 150 rocprofv3 --pmc $PMC --output-format csv -d $O/${T}_pmc_$N -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra > /dev/null 2> $O/${T}_pmc_$N.err || { echo "pmc $PMC failed"; tail $O/${T}_pmc_$N.err; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc $PMC --output-format csv -d $O/${T}a_pmc_$N -o run -- python3 bench.py --config anim120 --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $O/${T}a_pmc_$N.err || { echo "anim pmc $PMC failed"; tail $O/${T}a_pmc_$N.err; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_kt -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/${T}_bench_kt.json 2> $O/${T}_kt.err || { tail $O/${T}_kt.err; exit 1; }
for f in $O/${T}_bench*.json; do python3 -c "import json,sys;d=json.load(open('$f'));print('$f', d.get('config_name'), d['value'], d['ms_per_step'])"; done
echo session done
