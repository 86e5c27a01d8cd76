#!/usr/bin/env bash
# Round 5: the c2 regime test on the whole image; a finer back-claim sweep at 6 waves per SIMD (the
# share maps to dispatch rounds: 1536 blocks = 6 per CU, 50 % = the last three rounds).
set -euo pipefail
TAG=${1:-r05v}; OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    "tests/test_gpu_regime.py::test_c2_bench_regime_matches_oracle" > "$OUT/tests.log" 2>&1
tail -2 "$OUT/tests.log"
for r in 1 2 3; do
  for b in 33 40 45 50 20; do
    PT_MI355_CT_WAVES=6 PT_MI355_BACK=$b timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-configs4 > "$OUT/c2.json" 2>/dev/null
    echo "{\"back\": $b, \"ms\": $(python3 -c "import json;print(json.loads(open('$OUT/c2.json').read().strip().splitlines()[-1])['ms_per_step'])")}" >> "$OUT/ab.jsonl"
  done
done
python3 -c "
import json, collections
d = collections.defaultdict(list)
for l in open('$OUT/ab.jsonl'):
    x = json.loads(l); d[x['back']].append(x['ms'])
for k in sorted(d): print(k, [round(v, 4) for v in d[k]], round(sum(d[k]) / len(d[k]), 4))"
