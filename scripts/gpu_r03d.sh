#!/usr/bin/env bash
# GPU tests + headline benches + rocprofv3 evidence (c2 diffuse, v4) in one call.
set -euo pipefail
TAG=${1:-r03d}
bash scripts/gpu_r03c.sh "$TAG"
STEPS=10 bash scripts/round_profile.sh "$TAG" c2_1080p v4_1080p
