#!/usr/bin/env bash
# Round 5: the whole -m gpu suite on the tree, then the occupancy modes A/B (default = the per-geometry
# timing in ABBA order, against 5 and 6 waves per SIMD fixed).
set -euo pipefail
TAG=${1:-r05c}
bash scripts/gpu_tests.sh "$TAG"
VARIANTS="X=0|PT_MI355_CT_WAVES=5|PT_MI355_CT_WAVES=6" \
GEOS="1920 1080 8 8;3840 2160 8 8;3840 2160 64 8;1280 720 8 8;1920 1080 1 8" \
PT_QP_K=40 bash scripts/gpu_ab.sh "$TAG" 2
