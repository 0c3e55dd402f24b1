#!/bin/bash
# Round 6, session r09r: the f32 slab time as one fma (v_fmamk_f32) against the consolidation binary z;
# the culling edge tests (points kernel with f32 culling); VALU per wave of the 4K kernel; sphere steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r09r}
A=tinyraytracerinrust_amd/ab
N=tinyraytracerinrust_amd/librt_mi355x.so
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s tests/test_gpu_cull_edges.py tests/test_gpu_texel_boundary.py::test_texel_boundaries_headline_scene > $O/${T}_edges.txt 2>&1 || { tail -30 $O/${T}_edges.txt; exit 1; }
grep -E "points|passed|failed" $O/${T}_edges.txt
for C in globes4k sphere1080d0 globes1080d5; do
  timeout -k 10 300 python -u tools/ab_libs.py $A/librt_mi355x_z.so $N --config $C >> $O/${T}_ab.txt 2>&1 || { tail -20 $O/${T}_ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/${T}_ab.txt
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES --output-format csv -d $O/${T}_4k_pmc -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra > /dev/null 2> $O/${T}_4k_pmc.err || { tail $O/${T}_4k_pmc.err; exit 1; }
timeout -k 10 200 python -u bench.py --config sphere1080d0 --no-cpu-baseline > $O/${T}_sphere_bench.json 2> $O/${T}_sphere_bench.err || { tail $O/${T}_sphere_bench.err; exit 1; }
timeout -k 10 200 python -u bench.py --config sphere1080d0 --steps 50 --no-cpu-baseline > $O/${T}_sphere_bench50.json 2>> $O/${T}_sphere_bench.err || { tail $O/${T}_sphere_bench.err; exit 1; }
python3 -c "
import json
for f in ('$O/${T}_sphere_bench.json','$O/${T}_sphere_bench50.json'):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'], d['steps'], d.get('kernel_ms_mean'))"
echo session done
