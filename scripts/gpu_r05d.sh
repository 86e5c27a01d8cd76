#!/usr/bin/env bash
# Round 5: endgame item stealing in the continuous-tiles kernels -- the parity suites that exercise
# it first (any failure ends the call), then an interleaved A/B against the no-steal build.
set -euo pipefail
TAG=${1:-r05d}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_regime.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_state.py \
    > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
VARIANTS="X=0|PT_MI355_LIB=build/libpt_nosteal.so" \
GEOS="1920 1080 8 8;3840 2160 8 8;3840 2160 64 8;1280 720 8 8;1920 1080 1 8" \
PT_QP_K=40 bash scripts/gpu_ab.sh "$TAG" 3
