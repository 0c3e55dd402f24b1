# Pipeline GPU test; refraction kernel at 5 waves/SIMD (27 spilled VGPRs) vs 4 (product).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/r02bh_pytest.txt 2>&1 || { tail -30 $O/r02bh_pytest.txt; exit 1; }
tail -1 $O/r02bh_pytest.txt
for t in 0.1 0.6; do
timeout -k 10 300 python tools/ab_interleaved.py tinyraytracerinrust_amd/librt_mi355x.so tinyraytracerinrust_amd/build/librt_mi355x_refr5.so --reps 12 --burst 10 --size 1920x1080 --scene spinning_globes --time $t >> $O/r02bh_ab.txt 2>&1 || exit 1
done
grep -v amdgpu $O/r02bh_ab.txt
