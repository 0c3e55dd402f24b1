# Host culling switches across the bundled scenes (1080p, depth 10): oriented boxes off
# (RT_NO_OBB=1), draw-order walks (RT_DRAW_ORDER_SHADOWS=1), CSG literal order off
# (RT_NO_LIT_ORDER=1), each against HEAD, interleaved in one process per scene.
set -o pipefail
export TMPDIR=/tmp
P=tinyraytracerinrust_amd/librt_mi355x.so
for sc in fractal spinning_gimbals ground_star three_cubes spinning_cube; do
  timeout -k 10 300 python tools/ab_interleaved.py $P $P $P $P --upload-env - RT_NO_OBB=1 RT_DRAW_ORDER_SHADOWS=1 RT_NO_LIT_ORDER=1 \
    --reps 8 --burst 5 --size 1920x1080 --scene $sc --time 0.3 2>&1 | grep -v amdgpu || exit 1
done
