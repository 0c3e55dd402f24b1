# Full session: GPU tests, bench, probes, kernel trace, PMC passes, every BASELINE config line,
# then PMC passes of the anim120 config (refraction kernel).  Every GPU step has its own limit.
set -o pipefail
T=${TAG:-r02bi}
O=gpurun_out
TAG=$T PROBES=1 PMC_PASSES=1 bash tools/gpu_round2.sh && TAG=$T bash tools/gpu_configs.sh || exit 1
for PMC in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64" "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES"; do
  N=$(echo $PMC | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 120 rocprofv3 --pmc $PMC --output-format csv -d $O/${T}anim_pmc_$N -o run -- python3 bench.py --config anim120 --steps 1 --warmup 0 --settle-ms 0 --no-cpu-baseline > /dev/null 2> $O/${T}anim_pmc_$N.err || { echo "anim pmc pass $PMC failed"; exit 1; }
done
echo session done
