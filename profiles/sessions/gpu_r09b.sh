#!/bin/bash
# Round 6, session r09b: the primary-ray kernel (rt_spec_prim_*) -- the spec / fullsize GPU tests at the
# new binary, then interleaved A/B against the f32-cull binary (ab/librt_mi355x_f32.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r09b}
sha256sum tinyraytracerinrust_amd/librt_mi355x.so | cut -c1-16 > $O/${T}_so_sha16.txt
( while sleep 50; do date +%T >> $O/${T}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_spec_async.py tests/test_gpu_spec_family.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_pytest_gpu.txt 2>&1 || { tail -40 $O/${T}_pytest_gpu.txt; exit 1; }
tail -2 $O/${T}_pytest_gpu.txt
B=tinyraytracerinrust_amd/ab/librt_mi355x_f32.so
N=tinyraytracerinrust_amd/librt_mi355x.so
for C in sphere1080d0 globes4k; do
  timeout -k 10 300 python -u tools/ab_libs.py $B $N --config $C >> $O/${T}_ab.txt 2>&1 || { tail -20 $O/${T}_ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/${T}_ab.txt
timeout -k 10 300 python bench.py --config sphere1080d0 > $O/${T}_bench_sphere.json 2> $O/${T}_bench_sphere.err || { tail $O/${T}_bench_sphere.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/${T}_bench_sphere.json'));print('sphere bench', d['value'], d['ms_per_step'])"
echo session done
