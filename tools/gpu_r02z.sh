set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
for PMC in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES" "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64" "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  N=$(echo $PMC | tr ' ' '_' | cut -c1-30)
  timeout -s KILL 120 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d $O/r02z_anim_pmc_$N -o run -- python3 bench.py --config anim120 --steps 1 --warmup 0 --settle-ms 0 --no-cpu-baseline --streams 1 > /dev/null 2> $O/r02z.err || { tail $O/r02z.err; exit 1; }
done
echo done
