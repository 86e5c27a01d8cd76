#!/usr/bin/env bash
# Refresh the rocprofv3 evidence of every bench workload (run via gpurun from the repo root):
#   bash scripts/round_profile.sh TAG [workload ...]
# c2_1080p -> gpurun_out/prof/TAG, others -> gpurun_out/prof/TAG_<short>; then locally
#   python3 scripts/summarize_profile.py TAG c2_1080p   (etc.) writes profiles/.
set -euo pipefail
TAG=$1; shift
WLS=${*:-c2_1080p c3_4k c4_env_1080p v4_1080p}
for wl in $WLS; do
    case $wl in
        c2_1080p) t=$TAG ;;
        c3_4k) t=${TAG}_c3 ;;
        c4_env_1080p) t=${TAG}_c4 ;;
        v4_1080p) t=${TAG}_v4 ;;
        c5_8k) t=${TAG}_c5 ;;
        *) echo "unknown workload $wl"; exit 2 ;;
    esac
    echo "== $wl -> $t"
    WORKLOAD=$wl STEPS=${STEPS:-10} bash scripts/profile_gpu.sh "$t"
done
