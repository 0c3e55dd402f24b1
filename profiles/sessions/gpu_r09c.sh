#!/bin/bash
# Round 6, session r09c: (A) PMC of the 4K headline kernel at the f32-cull + primary-ray binary
# (instruction classes, FP64, HBM, issue), (B) its solo kernel trace, (C) anim120 traffic sweep:
# wave-pool slots (RT_SPEC_KP) and 32x2 tiles, bench value + FETCH / WRITE per variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r09c}
sha256sum tinyraytracerinrust_amd/librt_mi355x.so | cut -c1-16 > $O/${T}_so_sha16.txt
( while sleep 50; do date +%T >> $O/${T}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
if [ "${PMC4K:-1}" = "1" ]; then
for PMC in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64" "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES" "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32" "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH"; do
  N=$(echo $PMC | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 150 rocprofv3 --pmc $PMC --output-format csv -d $O/${T}_pmc_$N -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra > /dev/null 2> $O/${T}_pmc_$N.err || { echo "pmc $PMC failed"; tail $O/${T}_pmc_$N.err; exit 1; }
done
python3 tools/pmc_quick.py ${T}_pmc_ rt_spec_rows_00
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_kt -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/${T}_bench_kt.json 2> $O/${T}_kt.err || { tail $O/${T}_kt.err; exit 1; }
grep -i "spec_rows\|KernelName\|Name" $O/${T}_kt/run_kernel_stats.csv | head -5
fi
E=tinyraytracerinrust_amd/ab/librt_mi355x_env.so
T32=tinyraytracerinrust_amd/ab/librt_mi355x_t32.so
for V in ${VARIANTS:-env:122 env:250 env:314 t32:122 t32:250}; do
  L=$E; [ ${V%%:*} = t32 ] && L=$T32
  KP=${V##*:}
  TT=${T}_anim_${V%%:*}_${KP}
  RT_LIB_PATH=$L RT_SPEC_KP=$KP timeout -k 10 400 python bench.py --config anim120 --steps 3 --warmup 2 --no-cpu-baseline > $O/${TT}.json 2> $O/${TT}.err || { tail $O/${TT}.err; exit 1; }
  for PMC in FETCH_SIZE WRITE_SIZE; do
    RT_LIB_PATH=$L RT_SPEC_KP=$KP timeout -s KILL 240 rocprofv3 --pmc $PMC --output-format csv -d $O/${TT}_pmc_$PMC -o run -- python3 bench.py --config anim120 --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $O/${TT}_pmc_$PMC.err || { echo "anim pmc $PMC failed"; tail $O/${TT}_pmc_$PMC.err; exit 1; }
  done
  python3 -c "import json;d=json.load(open('$O/${TT}.json'));print('anim120 $V', d['value'], d['ms_per_step'])"
  python3 tools/pmc_quick.py ${TT}_pmc_ rt_spec_rows_00 | grep HBM
done
echo session done
