#!/usr/bin/env bash
# Round 5: back-claim share for the 6-wave env CT kernel (c4) and the 6-wave v4 CT kernel (1080p 8 spp).
set -euo pipefail
TAG=${1:-r05k}; OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
VARIANTS="X=0|PT_MI355_BACK=0|PT_MI355_BACK=33|PT_MI355_BACK=45|PT_MI355_BACK=60" \
GEOS="1920 1080 16 8 env;1920 1080 8 8 env" PT_QP_K=40 bash scripts/gpu_ab.sh "${TAG}_env" 2
export PT_QP_K=30
for r in 1 2; do
  for v in "X=0" "PT_MI355_BACK=0" "PT_MI355_BACK=33" "PT_MI355_BACK=45" "PT_MI355_BACK=60"; do
    line=$(env $v timeout -k 10 120 python3 scripts/v4_perf.py 1920 1080 8 8)
    echo "{\"variant\": \"$v\", \"r\": $line}" >> "$OUT/v4.jsonl"
  done
done
python3 - "$OUT/v4.jsonl" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    j = json.loads(line); r = j["r"]
    d[(r["W"], r["H"], r["spp"], j["variant"])].append("%.4f" % r["ms_per_launch"])
for k in sorted(d):
    print(k, d[k])
PY
