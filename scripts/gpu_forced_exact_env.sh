#!/usr/bin/env bash
# Parity of the certified texel cells' exact fallback (run via gpurun from the repo root): the library
# built with -DPT_EC_FORCE_EXACT=1 (build/libpt_fexact.so: no cell certified, every env lookup runs the
# glibc-exact atan2f/asinf branch) against the env, v4 and config tests.
set -euo pipefail
TAG=${1:-fexact}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp PT_MI355_LIB=$PWD/build/libpt_fexact.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py tests/test_gpu_v4.py tests/test_gpu_configs.py -m gpu -q \
    --timeout 120 --timeout-method thread -rf > "$OUT/fexact_tests.log" 2>&1 \
    || { tail -40 "$OUT/fexact_tests.log"; exit 1; }
tail -2 "$OUT/fexact_tests.log"
