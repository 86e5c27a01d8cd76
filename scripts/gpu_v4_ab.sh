#!/usr/bin/env bash
# Round 4 dev tool: v4 continuous-tiles kernel vs the per-tile one over geometries (scripts/v4_perf.py)
set -euo pipefail
TAG=${1:-v4ab}; ROUNDS=${2:-2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp PT_QP_K=30
for r in $(seq "$ROUNDS"); do
  for geo in "1920 1080 8 8" "1920 1080 1 8" "3840 2160 8 8" "1920 1080 32 8"; do
    timeout -k 10 120 python3 scripts/v4_perf.py $geo >> "$OUT/ab.jsonl"
    PT_MI355_NO_CT=1 timeout -k 10 120 python3 scripts/v4_perf.py $geo >> "$OUT/ab.jsonl"
  done
done
python3 - "$OUT/ab.jsonl" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    j = json.loads(line)
    d[(j["W"], j["H"], j["spp"], j["ct"])].append("%.4f/%.3f" % (j["ms_per_launch"], j["lane_eff"]))
for k in sorted(d):
    print(k, d[k])
PY
