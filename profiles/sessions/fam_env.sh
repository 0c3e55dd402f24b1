# family program: which in-process hipRTC compiles on the box come out large (diag build dumps)
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
D=tinyraytracerinrust_amd/build/librt_mi355x_dbg.so
O=gpurun_out
A="--scene spinning_globes --time 0.3 --size 1920x1080 --depth 10 --reps 3 --burst 1"
mkdir -p $O/r05v_A $O/r05v_B $O/r05v_C $O/r05v_D
RT_SPEC_DUMP_DIR=$O/r05v_A timeout -k 10 200 python -u tools/ab_interleaved.py $D --option 6=1 --family 1 $A > $O/r05v_A.txt 2>&1 || exit 1
RT_SPEC_DUMP_DIR=$O/r05v_B timeout -k 10 200 python -u tools/ab_interleaved.py $D $D --option 6=1 6=1 --family - 1 $A > $O/r05v_B.txt 2>&1 || exit 1
RT_SPEC_DUMP_DIR=$O/r05v_C timeout -k 10 200 rocprofv3 --kernel-trace -d $O/r05v_Ckt -o run -- python3 tools/ab_interleaved.py $D $D --option 6=1 6=1 --family - 1 $A > $O/r05v_C.txt 2>&1 || exit 1
RT_SPEC_DUMP_DIR=$O/r05v_D timeout -k 10 200 python -u tools/ab_interleaved.py $D --option 6=1 $A > $O/r05v_D.txt 2>&1 || exit 1
grep median $O/r05v_?.txt
