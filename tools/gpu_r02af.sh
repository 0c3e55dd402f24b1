set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_antialias.py tests/test_gpu_fastclamp.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/r02af_pytest.txt 2>&1 || { tail -40 $O/r02af_pytest.txt; exit 1; }
tail -2 $O/r02af_pytest.txt
timeout -k 10 200 python tools/aa_timing.py > $O/r02af_aa_timing.txt 2>&1 || { tail $O/r02af_aa_timing.txt; exit 1; }
RT_FAST_CLAMP=0 timeout -k 10 200 python tools/aa_timing.py >> $O/r02af_aa_timing.txt 2>&1 || exit 1
cat $O/r02af_aa_timing.txt
