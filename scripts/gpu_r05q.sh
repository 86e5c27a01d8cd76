#!/usr/bin/env bash
# Round 5: late split (PT_MI355_LATE_SPLIT=k: a whole tile claimed while its group has fewer than
# k/8 x its waves' count of units left runs as two halves, the second left for a wave whose queue is
# dry).  Parity with it on (regime / parity / config tests), then the c2 bench interleaved over k.
set -euo pipefail
TAG=${1:-r05q}; OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
PT_MI355_LATE_SPLIT=8 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_regime.py tests/test_gpu_parity.py tests/test_gpu_env.py > "$OUT/tests.log" 2>&1
tail -3 "$OUT/tests.log"
for r in 1 2; do
  for k in 0 2 4 8 16; do
    PT_MI355_LATE_SPLIT=$k timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-configs4 > "$OUT/c2.json" 2>/dev/null
    echo "{\"k\": $k, \"wl\": \"c2\", \"ms\": $(python3 -c "import json;print(json.loads(open('$OUT/c2.json').read().strip().splitlines()[-1])['ms_per_step'])")}" >> "$OUT/ab.jsonl"
  done
done
cat "$OUT/ab.jsonl"
