#!/bin/bash
# Round 5: RGBA8 frames that fit the L2s stored through the cache with the XCD-aware tile order
# (k_rows.hip RT_CACHED_FRAME_BYTES) against the previous product (b9114232): A/B time per frame on
# the three row configs, anim120 bench lines of both libraries, then the GPU suite on the new library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r08p}
P=tinyraytracerinrust_amd/librt_mi355x.so
V=tinyraytracerinrust_amd/build/librt_mi355x_prev.so
for C in globes4k globes1080d5 sphere1080d0; do
  timeout -k 10 300 python -u tools/ab_libs.py $V $P --config $C >> $O/${T}_cached_ab.txt 2>&1 || { tail -20 $O/${T}_cached_ab.txt; exit 1; }
done
cat $O/${T}_cached_ab.txt
run_anim() {   # name, env...
  local N=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config anim120 --steps 3 --warmup 2 --no-cpu-baseline > $O/${T}_anim_$N.json 2> $O/${T}_anim_$N.err || { tail $O/${T}_anim_$N.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/${T}_anim_$N.json'));print('anim $N', d['value'], d['ms_per_step'])"
}
run_anim prev RT_LIB_PATH=$V || exit 1
run_anim new RT_X=0 || exit 1
run_anim prev2 RT_LIB_PATH=$V || exit 1
run_anim new2 RT_X=0 || exit 1
timeout -k 10 300 python bench.py --config sphere1080d0 > $O/${T}_bench_sphere.json 2> $O/${T}_bench_sphere.err || { tail $O/${T}_bench_sphere.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/${T}_bench_sphere.json'));print('sphere', d['value'], d['ms_per_step'])"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_pytest_gpu.txt 2>&1 || { tail -40 $O/${T}_pytest_gpu.txt; exit 1; }
tail -2 $O/${T}_pytest_gpu.txt
echo session done
