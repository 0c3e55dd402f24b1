TAG=r01ah bash tools/gpu_round.sh || exit 1
for c in globes1080d5 sphere1080d0; do timeout -k 10 200 python bench.py --config $c --steps 40 --warmup 10 --no-cpu-baseline > gpurun_out/r01ah_bench_$c.json 2>gpurun_out/r01ah_c.err || exit 1; done
for k in 1 2 4; do timeout -k 10 200 python bench.py --config anim120 --steps 3 --warmup 1 --no-cpu-baseline --streams $k > gpurun_out/r01ah_bench_anim120_s$k.json 2>>gpurun_out/r01ah_c.err || exit 1; done
timeout -k 10 200 python tools/pipeline_probe.py > gpurun_out/r01ah_pipeline_probe.txt 2>&1
