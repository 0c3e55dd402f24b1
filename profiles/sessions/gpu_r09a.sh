#!/bin/bash
# Round 6, session r09a: f32 culling slab tests (RT_CULL_F32) -- the GPU suite at the new binary, then
# interleaved A/B against the round-5 binary (ab/librt_mi355x_base.so) on the BASELINE configs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r09a}
sha256sum tinyraytracerinrust_amd/librt_mi355x.so | cut -c1-16 > $O/${T}_so_sha16.txt
( while sleep 50; do date +%T >> $O/${T}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_pytest_gpu.txt 2>&1 || { tail -40 $O/${T}_pytest_gpu.txt; exit 1; }
  tail -2 $O/${T}_pytest_gpu.txt
fi
B=tinyraytracerinrust_amd/ab/librt_mi355x_base.so
N=tinyraytracerinrust_amd/librt_mi355x.so
for C in ${CONFIGS:-globes4k sphere1080d0 globes1080d5}; do
  timeout -k 10 300 python -u tools/ab_libs.py $B $N ${EXTRA_LIBS:-} --config $C >> $O/${T}_ab.txt 2>&1 || { tail -20 $O/${T}_ab.txt; exit 1; }
done
cat $O/${T}_ab.txt | grep -v amdgpu.ids
if [ "${ANIM:-1}" = "1" ]; then
  for L in $B $N; do
    RT_LIB_PATH=$L timeout -k 10 400 python bench.py --config anim120 --steps 3 --warmup 2 --no-cpu-baseline > $O/${T}_anim_$(basename $L .so).json 2> $O/${T}_anim_$(basename $L .so).err || { tail $O/${T}_anim_$(basename $L .so).err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${T}_anim_$(basename $L .so).json'));print('anim120 $L', d['value'], d['ms_per_step'])"
  done
fi
echo session done
