set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
L=tinyraytracerinrust_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r02g_pytest.txt 2>&1 || { tail -40 $O/r02g_pytest.txt; exit 1; }
tail -2 $O/r02g_pytest.txt
timeout -k 10 300 python tools/ab_interleaved.py $L/librt_mi355x.so $L/build/librt_mi355x_mega.so $L/build/librt_mi355x_ad8.so $L/build/librt_mi355x_ad6.so --reps 20 > $O/r02g_ab.txt 2>&1 || { tail $O/r02g_ab.txt; exit 1; }
timeout -k 10 300 python tools/ab_interleaved.py $L/librt_mi355x.so $L/build/librt_mi355x_mega.so --reps 20 --size 1920x1080 --depth 5 >> $O/r02g_ab.txt 2>&1 || { tail $O/r02g_ab.txt; exit 1; }
cat $O/r02g_ab.txt
timeout -k 10 300 python tools/inflight_probe.py $L/librt_mi355x.so $L/build/librt_mi355x_alldef.so > $O/r02g_inflight.txt 2>&1 || { tail $O/r02g_inflight.txt; exit 1; }
cat $O/r02g_inflight.txt
