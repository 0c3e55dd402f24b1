# PMC passes of the anim120 config (the refraction kernel), one rocprofv3 run per counter group.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
TAG=r02ao
for PMC in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64" "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES" "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY" "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES"; do
  N=$(echo $PMC | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 120 rocprofv3 --pmc $PMC --output-format csv -d $O/${TAG}_pmc_$N -o run -- python3 bench.py --config anim120 --steps 1 --warmup 0 --settle-ms 0 --no-cpu-baseline > /dev/null 2> $O/${TAG}_pmc_$N.err || { echo "pmc pass $PMC failed (see $O/${TAG}_pmc_$N.err)"; tail -5 $O/${TAG}_pmc_$N.err; exit 1; }
done
echo done
