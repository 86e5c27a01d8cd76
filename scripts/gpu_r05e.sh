#!/usr/bin/env bash
# Round 5: what the stealing build's slowdown is made of -- the structure alone (nopub: victims never
# publish), longer waits (sleep16), against the no-steal build and the default.
set -euo pipefail
VARIANTS="X=0|PT_MI355_LIB=build/libpt_nosteal.so|PT_MI355_LIB=build/libpt_nopub.so|PT_MI355_LIB=build/libpt_sleep16.so" \
GEOS="1920 1080 8 8;3840 2160 64 8;1280 720 8 8" \
PT_QP_K=40 bash scripts/gpu_ab.sh ${1:-r05e} 2
