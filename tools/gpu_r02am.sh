# A/B: concentric sphere leaves sharing their ray terms (RT_SPHERE_SHARE), interleaved in one
# process; then the parity tests on the product library.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
B=tinyraytracerinrust_amd/build
P=tinyraytracerinrust_amd/librt_mi355x.so
timeout -k 10 300 python tools/ab_interleaved.py $B/librt_mi355x_base.so $B/librt_mi355x_noshare.so $P --reps 12 --burst 10 > $O/r02am_ab.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab_interleaved.py $B/librt_mi355x_base.so $B/librt_mi355x_noshare.so $P --reps 12 --burst 10 --size 1920x1080 --scene spinning_globes --time 0.3 >> $O/r02am_ab.txt 2>&1 || exit 1
cat $O/r02am_ab.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fastclamp.py tests/test_gpu_deferred.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/r02am_pytest.txt 2>&1 || { tail -30 $O/r02am_pytest.txt; exit 1; }
tail -3 $O/r02am_pytest.txt
