#!/bin/bash
# Round 6, session r09f: (A) the tree-mode resource guard (verdict item 5): ray-tree programs at
# 1.4 KB/lane of scratch against the generic kernels (fuzz seed 11, a small glass-and-mirror scene);
# (B) PC sampling (host trap) of the 4K headline kernel, to attribute its time by instruction.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r09f}
sha256sum tinyraytracerinrust_amd/librt_mi355x.so | cut -c1-16 > $O/${T}_so_sha16.txt
( while sleep 50; do date +%T >> $O/${T}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
for SC in fuzz:11 profiles/sessions/tree_small.scene; do
  for D in 10 3; do
    timeout -k 10 300 python -u tools/spec_vs_generic.py $SC 1920x1080 0 $D 10 5 2>&1 | grep -v amdgpu.ids >> $O/${T}_tree_guard.txt || { tail $O/${T}_tree_guard.txt; exit 1; }
  done
done
cat $O/${T}_tree_guard.txt
timeout -k 10 400 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 --output-format csv -d $O/${T}_pcs -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra > $O/${T}_pcs_bench.json 2> $O/${T}_pcs.err || { echo "pc sampling failed"; tail -20 $O/${T}_pcs.err; exit 1; }
ls -la $O/${T}_pcs/ | head
echo session done
