#!/usr/bin/env bash
# Round 5: v4 GPU tests with the 6-wave continuous-tiles kernel (the default at 1080p 8 spp now), then
# the c2 tail policies re-tuned for the 6-wave grid (back-claim share, split factor).
set -euo pipefail
TAG=${1:-r05h}; OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_v4.py tests/test_gpu_flags.py tests/test_gpu_regime.py > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
VARIANTS="PT_MI355_CT_WAVES=6|PT_MI355_CT_WAVES=6 PT_MI355_BACK=0|PT_MI355_CT_WAVES=6 PT_MI355_BACK=33|PT_MI355_CT_WAVES=6 PT_MI355_BACK=45|PT_MI355_CT_WAVES=6 PT_MI355_SPLIT=2" \
GEOS="1920 1080 8 8" PT_QP_K=60 bash scripts/gpu_ab.sh "$TAG" 3
