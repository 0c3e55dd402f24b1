set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
L=tinyraytracerinrust_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r02f_pytest.txt 2>&1 || { tail -40 $O/r02f_pytest.txt; exit 1; }
tail -2 $O/r02f_pytest.txt
timeout -k 10 300 python tools/inflight_probe.py $L/librt_mi355x.so $L/build/librt_mi355x_mega.so > $O/r02f_inflight.txt 2>&1 || { tail $O/r02f_inflight.txt; exit 1; }
cat $O/r02f_inflight.txt
for K in 1.0 2.0 3.0; do RT_SPLIT_K=$K RT_DEFERRED=1 timeout -k 10 200 python tools/rank_share_probe.py $L/librt_mi355x.so >> $O/r02f_split_k.txt 2>&1 || exit 1; echo "K=$K" >> $O/r02f_split_k.txt; done
cat $O/r02f_split_k.txt
