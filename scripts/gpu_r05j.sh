#!/usr/bin/env bash
# Round 5: the env continuous-tiles kernel at 6 waves per SIMD (96-entry miss queues) and the 3-arm
# per-geometry timing (5 / 6 waves, 6 waves + 45 % back claims): parity suites, then A/B.
set -euo pipefail
TAG=${1:-r05j}; OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_env.py tests/test_gpu_regime.py tests/test_gpu_configs.py tests/test_gpu_parity.py \
    tests/test_gpu_output.py tests/test_gpu_flags.py > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
VARIANTS="X=0|PT_MI355_LIB=build/libpt_env5.so" \
GEOS="1920 1080 16 8 env;1920 1080 8 8 env;3840 2160 8 8 env" PT_QP_K=40 bash scripts/gpu_ab.sh "${TAG}_env" 2
VARIANTS="X=0|PT_MI355_CT_WAVES=5|PT_MI355_CT_WAVES=6" \
GEOS="1920 1080 8 8;3840 2160 8 8;1280 720 8 8;3840 2160 64 8;1920 1080 16 8" PT_QP_K=40 bash scripts/gpu_ab.sh "$TAG" 2
