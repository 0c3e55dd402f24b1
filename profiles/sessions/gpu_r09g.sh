#!/bin/bash
# Round 6, session r09g: the inside test's certain-outside fast path and the Lambert ratio through
# div_core: the GPU suite at the new binary, the texel-boundary and f64 bit-equality tests (printed),
# then interleaved A/B of HEAD (h2), the product, the product without the texel guard (tg0) and at 5 waves/SIMD (w5).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r09g}
sha256sum tinyraytracerinrust_amd/librt_mi355x.so | cut -c1-16 > $O/${T}_so_sha16.txt
( while sleep 50; do date +%T >> $O/${T}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_texel_boundary.py > $O/${T}_pytest_gpu.txt 2>&1 || { tail -40 $O/${T}_pytest_gpu.txt; exit 1; }
  tail -2 $O/${T}_pytest_gpu.txt
fi
timeout -k 10 600 python -u -m pytest tests/test_gpu_texel_boundary.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/${T}_texel.txt 2>&1 || { tail -40 $O/${T}_texel.txt; exit 1; }
grep -E "texel-boundary|bit-equal|passed|failed" $O/${T}_texel.txt
A=tinyraytracerinrust_amd/ab
N=tinyraytracerinrust_amd/librt_mi355x.so
for C in ${CONFIGS:-globes4k globes1080d5 sphere1080d0}; do
  timeout -k 10 300 python -u tools/ab_libs.py $A/librt_mi355x_h2.so $N $A/librt_mi355x_tg0.so $A/librt_mi355x_w5.so --config $C >> $O/${T}_ab.txt 2>&1 || { tail -20 $O/${T}_ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/${T}_ab.txt
for L in $A/librt_mi355x_h2.so $N; do
  B=$(basename $L .so)
  RT_LIB_PATH=$L timeout -k 10 400 python bench.py --config anim120 --steps 3 --warmup 2 --no-cpu-baseline > $O/${T}_anim_$B.json 2> $O/${T}_anim_$B.err || { tail $O/${T}_anim_$B.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/${T}_anim_$B.json'));print('anim120 $B', d['value'], d['ms_per_step'])"
done
echo session done
