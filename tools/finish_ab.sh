#!/bin/bash
# Wavefront path: small levels finished by the per-lane trace (RT_WF_FINISH = ray-count threshold;
# temporary A/B switch), fractal 1080p d10 lone frame, plus the wavefront parity tests at one setting.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out
for f in 0 16384 32768 65536 131072 262144 600000; do
  RT_WF_FINISH=$f timeout -k 10 120 python -u tools/scene_timing.py fractal 1920x1080 0 10 wavefront 4 2>&1 | grep -v amdgpu.ids | sed "s/^/finish<$f /" || exit 1
done
RT_WF_FINISH=${TESTF:-65536} timeout -k 10 300 python -u -m pytest tests/test_gpu_wavefront.py -x -q --timeout 120 --timeout-method thread > $O/finish_wf_tests.txt 2>&1 || { tail -30 $O/finish_wf_tests.txt; exit 1; }
tail -1 $O/finish_wf_tests.txt
