#!/usr/bin/env bash
# Parity of the closest-sphere stages' sequential fallbacks (run via gpurun from the repo root): the
# library built with -DPT_SPHERE_FORCE_SEQ=1 -DPT_V4_SPHERE_FORCE_SEQ=1 (build/libpt_fseq.so, every
# candidate ray takes the sequential tests) against the parity, v4 and config tests.  The fallback-
# RATE assertions are skipped (PT_TEST_FORCED_FALLBACK=1): 100 % by construction.
set -euo pipefail
TAG=${1:-fseq}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp PT_MI355_LIB=$PWD/build/libpt_fseq.so PT_TEST_FORCED_FALLBACK=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_v4.py tests/test_gpu_configs.py -m gpu -q \
    --timeout 120 --timeout-method thread -rf > "$OUT/fseq_tests.log" 2>&1 \
    || { tail -40 "$OUT/fseq_tests.log"; exit 1; }
tail -2 "$OUT/fseq_tests.log"
