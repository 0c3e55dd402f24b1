set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r02b_pytest.txt 2>&1 || { tail -40 $O/r02b_pytest.txt; exit 1; }
tail -2 $O/r02b_pytest.txt
L=tinyraytracerinrust_amd
timeout -k 10 300 python tools/ab_interleaved.py $L/librt_mi355x.so $L/build/librt_mi355x_def7.so $L/build/librt_mi355x_def6.so $L/build/librt_mi355x_mega.so --reps 20 > $O/r02b_ab4k.txt 2>&1 || { tail $O/r02b_ab4k.txt; exit 1; }
timeout -k 10 300 python tools/ab_interleaved.py $L/librt_mi355x.so $L/build/librt_mi355x_def7.so $L/build/librt_mi355x_mega.so --reps 20 --size 1920x1080 --depth 5 >> $O/r02b_ab4k.txt 2>&1 || { tail $O/r02b_ab4k.txt; exit 1; }
cat $O/r02b_ab4k.txt
timeout -k 10 300 python tools/rank_share_probe.py $L/librt_mi355x.so $L/build/librt_mi355x_mega.so > $O/r02b_rank_share.txt 2>&1 || { tail $O/r02b_rank_share.txt; exit 1; }
cat $O/r02b_rank_share.txt
