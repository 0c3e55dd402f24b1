set -o pipefail
cd "${GRAFT_REPO_ROOT}"
L=tinyraytracerinrust_amd/build/librt_mi355x_etimes.so
for cfg in "RT_DIAG_HOT=0" "RT_DIAG_HOT=64" "RT_DIAG_HOT=512" "RT_DIAG_HOT=2048" "RT_DIAG_GRID=64" "RT_DIAG_GRID=512" "RT_DIAG_GRID=2048"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python -u tools/entry_times_probe.py $L --world 8 2>&1 | grep -v amdgpu.ids | head -9 || exit 1
done
