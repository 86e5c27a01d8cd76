#!/usr/bin/env bash
# Round 5: the back-claim share over a wider range (c2 at 6 and 5 waves per SIMD, 4K 8 spp, 720p), and
# the env continuous-tiles kernel at 6 waves per SIMD with a smaller miss queue (c4).
set -euo pipefail
TAG=${1:-r05i}
VARIANTS="PT_MI355_CT_WAVES=6|PT_MI355_CT_WAVES=6 PT_MI355_BACK=45|PT_MI355_CT_WAVES=6 PT_MI355_BACK=55|PT_MI355_CT_WAVES=6 PT_MI355_BACK=70|PT_MI355_CT_WAVES=6 PT_MI355_BACK=90|PT_MI355_CT_WAVES=5|PT_MI355_CT_WAVES=5 PT_MI355_BACK=45|PT_MI355_CT_WAVES=5 PT_MI355_BACK=70" \
GEOS="1920 1080 8 8;3840 2160 8 8;1280 720 8 8" PT_QP_K=40 bash scripts/gpu_ab.sh "$TAG" 2
VARIANTS="X=0|PT_MI355_LIB=build/libpt_env6q96.so|PT_MI355_LIB=build/libpt_env6q64.so|PT_MI355_BACK=45|PT_MI355_BACK=70" \
GEOS="1920 1080 16 8 env;1920 1080 8 8 env" PT_QP_K=40 bash scripts/gpu_ab.sh "${TAG}_env" 2
