set -o pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out
for hl in "0 0" "1 0" "1 1" "1 2" "0 2"; do set -- $hl
  RT_WFP_HSORT=$1 RT_WFP_LSORT=$2 timeout -k 10 200 python -u tools/scene_timing.py fractal 1920x1080 0 10 wavefront:p5,wavefront:p1 4 2>/dev/null | sed "s/^/H$1 L$2 /" || exit 1
done
RT_WFP_HSORT=1 RT_WFP_LSORT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_wavefront.py -x -q --timeout 120 --timeout-method thread -k "parity or shells or overflow" > $O/r03o_wf_tests_h1l1.txt 2>&1 || { tail -30 $O/r03o_wf_tests_h1l1.txt; exit 1; }
tail -1 $O/r03o_wf_tests_h1l1.txt
