#!/usr/bin/env bash
# Round 5: 7 and 8 waves per SIMD for the diffuse continuous-tiles kernel (the pool loop needs no
# more than 72 / 64 VGPRs -- its spills are in the event code) against 5 and 6.
set -euo pipefail
VARIANTS="PT_MI355_CT_WAVES=5|PT_MI355_CT_WAVES=6|PT_MI355_CT_WAVES=6 PT_MI355_LIB=build/libpt_wide7.so|PT_MI355_CT_WAVES=6 PT_MI355_LIB=build/libpt_wide8.so" \
GEOS="1920 1080 8 8;3840 2160 64 8;3840 2160 8 8;1280 720 8 8" \
PT_QP_K=40 bash scripts/gpu_ab.sh ${1:-r05f} 2
