# scene-family timing probe: the family program alone, after an exact one, and under a kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
M=tinyraytracerinrust_amd/librt_mi355x.so
O=gpurun_out
A="--scene spinning_globes --time 0.3 --size 1920x1080 --depth 10"
timeout -k 10 200 python -u tools/ab_interleaved.py $M --option 6=1 --family 120 $A --reps 20 --burst 4 > $O/r05o_a.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab_interleaved.py $M $M --option 6=1 6=1 --family 120 - $A --reps 20 --burst 4 > $O/r05o_b.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab_interleaved.py $M $M --option 6=1 6=1 --family - 120 $A --reps 20 --burst 1 > $O/r05o_c.txt 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r05o_kt -o run -- python3 tools/ab_interleaved.py $M $M --option 6=1 6=1 --family - 120 $A --reps 10 --burst 4 > $O/r05o_d.txt 2>&1 || exit 1
cat $O/r05o_a.txt $O/r05o_b.txt $O/r05o_c.txt $O/r05o_d.txt | grep -v amdgpu.ids
