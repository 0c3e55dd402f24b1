set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
L=tinyraytracerinrust_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r02ac_pytest.txt 2>&1 || { tail -40 $O/r02ac_pytest.txt; exit 1; }
tail -2 $O/r02ac_pytest.txt
timeout -k 10 300 python tools/ab_interleaved.py $L/librt_mi355x.so $L/build/librt_mi355x_nofc.so --reps 12 --burst 10 > $O/r02ac_ab.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab_interleaved.py $L/librt_mi355x.so $L/build/librt_mi355x_nofc.so --reps 12 --burst 10 --size 1920x1080 --depth 5 >> $O/r02ac_ab.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab_interleaved.py $L/librt_mi355x.so $L/build/librt_mi355x_nofc.so --reps 12 --burst 10 --size 1920x1080 --scene spinning_globes --time 0.25 >> $O/r02ac_ab.txt 2>&1 || exit 1
cat $O/r02ac_ab.txt
