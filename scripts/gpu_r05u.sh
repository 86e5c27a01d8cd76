#!/usr/bin/env bash
# Round 5: the strengthened output / regime tests (whole images against the oracle; presenting vs
# plain accumulators at every occupancy).
set -euo pipefail
TAG=${1:-r05u}; OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_output.py tests/test_gpu_regime.py > "$OUT/tests.log" 2>&1
tail -3 "$OUT/tests.log"
grep -E "PASSED|FAILED" "$OUT/tests.log" | sed -E 's/.*::(\S+) (PASSED|FAILED).*/\1 \2/' | head -40
