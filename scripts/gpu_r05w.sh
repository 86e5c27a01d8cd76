#!/usr/bin/env bash
# Round 5, late: the tree's whole -m gpu suite and smoke(), then the finer back-claim sweep at 6 waves
# per SIMD (scripts/gpu_r05v.sh without its test).
set -euo pipefail
TAG=${1:-r05w}; OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf -p no:cacheprovider > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
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
