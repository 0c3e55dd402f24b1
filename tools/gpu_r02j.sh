set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r02j_pytest.txt 2>&1 || { tail -40 $O/r02j_pytest.txt; exit 1; }
tail -2 $O/r02j_pytest.txt
export RT_TILE_ORDER_DEBUG=1
TAG=r02j bash tools/gpu_configs.sh 2>&1 | cut -c1-400
grep -h "tile order" $O/r02j_bench_*.err
timeout -k 10 300 python tools/inflight_probe.py tinyraytracerinrust_amd/librt_mi355x.so > $O/r02j_inflight.txt 2>&1 || { tail $O/r02j_inflight.txt; exit 1; }
cat $O/r02j_inflight.txt | grep -v "^tile order"
grep "tile order" $O/r02j_inflight.txt | sort | uniq -c | head
