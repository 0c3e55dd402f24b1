# Oriented object boxes in the refraction kernels too (RT_OBB_REFR=1, obbr) vs HEAD: A/B on the
# refraction scenes, parity of obbr.
set -o pipefail
export TMPDIR=/tmp
B=tinyraytracerinrust_amd/build
P=tinyraytracerinrust_amd/librt_mi355x.so
timeout -k 10 300 python tools/ab_interleaved.py $P $B/librt_mi355x_obbr.so --reps 12 --burst 10 --size 1920x1080 --scene spinning_globes --time 0.3 2>&1 | grep -v amdgpu
timeout -k 10 300 python tools/ab_interleaved.py $P $B/librt_mi355x_obbr.so --reps 4 --burst 2 --size 1920x1080 --scene fractal --time 0.3 2>&1 | grep -v amdgpu
RT_LIB_PATH=$B/librt_mi355x_obbr.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread -m gpu 2>&1 | tail -1
