# rt_acos through the in-range sqrt / division cores (RT_ACOS_CORES) vs plain (ac0), full GPU suite.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
B=tinyraytracerinrust_amd/build
P=tinyraytracerinrust_amd/librt_mi355x.so
L="$B/librt_mi355x_ac0.so $P"
timeout -k 10 300 python tools/ab_interleaved.py $L --reps 15 --burst 10 > $O/r02cd_ab.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab_interleaved.py $L --reps 15 --burst 10 --depth 0 >> $O/r02cd_ab.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab_interleaved.py $L --reps 15 --burst 10 --size 1920x1080 --depth 5 >> $O/r02cd_ab.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab_interleaved.py $L --reps 15 --burst 10 --size 1920x1080 --scene spinning_globes --time 0.3 >> $O/r02cd_ab.txt 2>&1 || exit 1
grep -v amdgpu $O/r02cd_ab.txt
timeout -k 10 1000 python -u -m pytest tests -x -q --timeout 400 --timeout-method thread -m gpu > $O/r02cd_pytest.txt 2>&1 || { tail -30 $O/r02cd_pytest.txt; exit 1; }
tail -1 $O/r02cd_pytest.txt
timeout -k 10 300 python bench.py > $O/r02cd_bench.json 2> $O/r02cd_bench.err || exit 1; cat $O/r02cd_bench.json
