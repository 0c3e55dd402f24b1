# Full session: GPU tests, bench, probes, kernel trace, PMC passes, then every BASELINE config line.
set -o pipefail
TAG=${TAG:-r02bi} PROBES=1 PMC_PASSES=1 bash tools/gpu_round2.sh && TAG=${TAG:-r02bi} bash tools/gpu_configs.sh
