set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
M=tinyraytracerinrust_amd/librt_mi355x.so
O=gpurun_out
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_BRANCH"
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/r05n_exact -o run -- python3 tools/ab_interleaved.py $M --option 6=1 --scene spinning_globes --time 0.3 --size 1920x1080 --reps 3 > $O/r05n_exact.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/r05n_fam -o run -- python3 tools/ab_interleaved.py $M --option 6=1 --family 120 --scene spinning_globes --time 0.3 --size 1920x1080 --reps 3 > $O/r05n_fam.log 2>&1 || exit 1
echo done
