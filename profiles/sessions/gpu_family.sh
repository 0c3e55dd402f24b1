#!/bin/bash
# Scene families (rt_spec_family_register) and the specialised kernels compiled by the ROCm
# installation's hipRTC (spec.hip rtc()): the spec / family GPU tests, interleaved timing of one
# spinning_globes frame and of the 4K globes frame, and the bench lines (headline, anim120 with and
# without specialisation, globes1080d5).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r05w}
M=tinyraytracerinrust_amd/librt_mi355x.so
R3=tinyraytracerinrust_amd/build/librt_mi355x_r3.so
( while sleep 50; do date +%T >> $O/${T}_heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_spec_family.py tests/test_gpu_spec.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/${T}_pytest.txt 2>&1 || { tail -40 $O/${T}_pytest.txt; exit 1; }
tail -2 $O/${T}_pytest.txt
timeout -k 10 400 python -u tools/ab_interleaved.py $M $M $M --option 6=1 6=1 - --family - 120 - --scene spinning_globes --time 0.3 --size 1920x1080 --depth 10 --reps 30 --burst 4 --check > $O/${T}_ab_sg.txt 2>&1 || { tail -20 $O/${T}_ab_sg.txt; exit 1; }
grep -v amdgpu.ids $O/${T}_ab_sg.txt
timeout -k 10 400 python -u tools/ab_interleaved.py $M $M --option 6=1 - --reps 30 --burst 4 --check > $O/${T}_ab_4k.txt 2>&1 || { tail -20 $O/${T}_ab_4k.txt; exit 1; }
grep -v amdgpu.ids $O/${T}_ab_4k.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/${T}_bench.json 2> $O/${T}_bench.err || { tail $O/${T}_bench.err; exit 1; }
cat $O/${T}_bench.json
timeout -k 10 400 python bench.py --config anim120 --steps 3 --warmup 1 > $O/${T}_bench_anim120.json 2> $O/${T}_bench_anim120.err || { tail $O/${T}_bench_anim120.err; exit 1; }
cat $O/${T}_bench_anim120.json
timeout -k 10 300 python bench.py --config globes1080d5 --steps 20 --warmup 2 > $O/${T}_bench_globes1080d5.json 2> $O/${T}_bench_globes1080d5.err || { tail $O/${T}_bench_globes1080d5.err; exit 1; }
cat $O/${T}_bench_globes1080d5.json
echo session done
