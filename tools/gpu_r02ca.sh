# Occluder-first shadow rays (RT_SHADOW_HINT) A/B: HEAD-equivalent (h0), product (hint in a VGPR),
# hint in LDS (hlds), the any-hit walk with no hint (hnull).  Then parity of the product.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
B=tinyraytracerinrust_amd/build
P=tinyraytracerinrust_amd/librt_mi355x.so
L="$B/librt_mi355x_h0.so $P $B/librt_mi355x_hlds.so $B/librt_mi355x_hnull.so"
timeout -k 10 300 python tools/ab_interleaved.py $L --reps 12 --burst 10 > $O/r02ca_ab.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab_interleaved.py $L --reps 12 --burst 10 --depth 0 >> $O/r02ca_ab.txt 2>&1 || exit 1
RT_DEFERRED=0 timeout -k 10 300 python tools/ab_interleaved.py $L --reps 12 --burst 10 --size 1920x1080 --depth 5 >> $O/r02ca_ab.txt 2>&1 || exit 1
grep -v amdgpu $O/r02ca_ab.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/r02ca_pytest.txt 2>&1 || { tail -30 $O/r02ca_pytest.txt; exit 1; }
tail -1 $O/r02ca_pytest.txt
