# Lazy inside test (only for hits that may spawn a ray): A/B against HEAD, parity subset.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
B=tinyraytracerinrust_amd/build
P=tinyraytracerinrust_amd/librt_mi355x.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deferred.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/r02at_pytest.txt 2>&1 || { tail -30 $O/r02at_pytest.txt; exit 1; }
tail -1 $O/r02at_pytest.txt
timeout -k 10 300 python tools/ab_interleaved.py $B/librt_mi355x_head.so $P --reps 12 --burst 10 > $O/r02at_ab.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab_interleaved.py $B/librt_mi355x_head.so $P --reps 12 --burst 10 --size 1920x1080 --scene spinning_globes --time 0.3 >> $O/r02at_ab.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab_interleaved.py $B/librt_mi355x_head.so $P --reps 12 --burst 10 --size 1920x1080 --depth 5 >> $O/r02at_ab.txt 2>&1 || exit 1
cat $O/r02at_ab.txt
