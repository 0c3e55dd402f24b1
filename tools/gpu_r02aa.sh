set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -s KILL 60 rocprofv3 -L > $O/r02aa_counters.txt 2>&1 || true
grep -o "SQ_INSTS_VALU[A-Z0-9_]*" $O/r02aa_counters.txt | sort -u > $O/r02aa_valu_counters.txt || true
cat $O/r02aa_valu_counters.txt | tr '\n' ' '
echo
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 --output-format csv -d $O/r02aa_mix_pmc_a -o run -- python3 tools/render_loop.py 5 > /dev/null 2> $O/r02aa.err || { tail $O/r02aa.err; exit 1; }
echo done
