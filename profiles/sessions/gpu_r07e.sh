#!/bin/bash
# Round 5: completion events bound to the dispatch (A/B against no events), anim120 LDS-frame sweep
# with its HBM traffic.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r07e}
P=tinyraytracerinrust_amd/librt_mi355x.so
NM=tinyraytracerinrust_amd/build/librt_mi355x_nomarks.so
KLL=tinyraytracerinrust_amd/build/librt_mi355x_kl.so
for C in sphere1080d0 globes1080d5 globes4k; do
  timeout -k 10 300 python -u tools/ab_libs.py $P $NM --config $C >> $O/${T}_marks_ab.txt 2>&1 || { tail -20 $O/${T}_marks_ab.txt; exit 1; }
done
cat $O/${T}_marks_ab.txt
for KL in 1 2 3 4 5; do
  RT_LIB_PATH=$KLL RT_SPEC_KL=$KL timeout -k 10 300 python bench.py --config anim120 --steps 10 --warmup 2 --no-cpu-baseline > $O/${T}_anim_kl$KL.json 2> $O/${T}_anim_kl$KL.err || { tail $O/${T}_anim_kl$KL.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/${T}_anim_kl$KL.json'));print('KL $KL', d['value'], d['ms_per_step'], d['roofline']['kernel'][:150])"
done
for KL in 2 3 5; do
  for PMC in FETCH_SIZE WRITE_SIZE; do
    RT_LIB_PATH=$KLL RT_SPEC_KL=$KL timeout -s KILL 240 rocprofv3 --pmc $PMC --output-format csv -d $O/${T}a_kl${KL}_$PMC -o run -- python3 bench.py --config anim120 --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $O/${T}a_kl${KL}_$PMC.err || { echo "pmc $KL $PMC failed"; tail $O/${T}a_kl${KL}_$PMC.err; exit 1; }
  done
done
echo session done
