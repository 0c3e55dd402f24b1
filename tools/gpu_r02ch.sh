# Oriented object boxes (RT_OBB) vs world boxes only (obb0): A/B, event counts, whole GPU suite.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
B=tinyraytracerinrust_amd/build
P=tinyraytracerinrust_amd/librt_mi355x.so
L="$B/librt_mi355x_obb0.so $P"
timeout -k 10 300 python tools/ab_interleaved.py $L --reps 15 --burst 10 > $O/r02ch_ab.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab_interleaved.py $L --reps 15 --burst 10 --depth 0 >> $O/r02ch_ab.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab_interleaved.py $L --reps 15 --burst 10 --size 1920x1080 --depth 5 >> $O/r02ch_ab.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab_interleaved.py $L --reps 15 --burst 10 --size 1920x1080 --scene spinning_globes --time 0.3 >> $O/r02ch_ab.txt 2>&1 || exit 1
grep -v amdgpu $O/r02ch_ab.txt
timeout -k 10 1000 python -u -m pytest tests -x -q --timeout 400 --timeout-method thread -m gpu > $O/r02ch_pytest.txt 2>&1 || { tail -30 $O/r02ch_pytest.txt; exit 1; }
tail -1 $O/r02ch_pytest.txt
