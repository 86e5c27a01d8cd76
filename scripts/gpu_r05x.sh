#!/usr/bin/env bash
# Round 5: the output-stage tests (the full-size env present check added).
set -euo pipefail
TAG=${1:-r05x}; OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_output.py > "$OUT/tests.log" 2>&1
tail -3 "$OUT/tests.log"
