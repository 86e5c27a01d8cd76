#!/usr/bin/env bash
# Round 5: interleaved A/B -- the slot area's fabric traffic (timing-only alias build, wrong images)
# and the per-geometry 5/6-waves timing (PT_MI355_CT_WAVES=0) against the default.
set -euo pipefail
VARIANTS="X=0|PT_MI355_LIB=build/libpt_alias.so|PT_MI355_CT_WAVES=0" \
GEOS="1920 1080 8 8;1920 1080 16 8 env;3840 2160 8 8;3840 2160 64 8;1280 720 8 8" \
PT_QP_K=40 bash scripts/gpu_ab.sh ${1:-r05b} 3
