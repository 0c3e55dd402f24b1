# PMC passes of the product render kernels, RT_DEFERRED=0 (megakernel) vs 1 (deferred shadows),
# 4K globes d10, one pass per counter group, each under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out
TAG=${TAG:-r02e}
for V in 0 1; do
  for PMC in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU" "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64"; do
    N=$(echo $PMC | tr ' ' '_' | cut -c1-30)
    RT_DEFERRED=$V timeout -s KILL 90 rocprofv3 --pmc $PMC --output-format csv -d $O/${TAG}_d${V}_pmc_$N -o run -- python3 tools/render_loop.py 5 > /dev/null 2> $O/${TAG}_d${V}_pmc_$N.err || { echo "pmc pass $V $PMC failed"; tail -5 $O/${TAG}_d${V}_pmc_$N.err; exit 1; }
  done
done
echo done
