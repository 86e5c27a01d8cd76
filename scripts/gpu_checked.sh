#!/usr/bin/env bash
# The -m gpu suite under the bounds-checked build (build/libpt_checked.so, PT_CHECKED=1: pt_guard.h),
# once: every guard of the continuous-tiles pools and the schedule builder must stay silent.
set -euo pipefail
TAG=${1:-checked}; OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
PT_MI355_LIB=build/libpt_checked.so timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 \
    --timeout-method thread -rfs -p no:cacheprovider > "$OUT/gpu_tests_checked.log" 2>&1 || { tail -60 "$OUT/gpu_tests_checked.log"; exit 1; }
tail -3 "$OUT/gpu_tests_checked.log"
