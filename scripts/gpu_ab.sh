#!/usr/bin/env bash
# Dev tool: interleaved A/B of library settings (env-var variants) with scripts/quick_perf.py.
#   VARIANTS="A=1|A=0 B=2" GEOS="1920 1080 8 8;3840 2160 8 8" bash scripts/gpu_ab.sh TAG ROUNDS
# TESTS="pytest args" runs those -m gpu tests first.  Output: gpurun_out/TAG/ab.jsonl + a summary.
set -euo pipefail
TAG=${1:-ab}; ROUNDS=${2:-2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp PT_QP_K=${PT_QP_K:-60}
if [ -n "${TESTS:-}" ]; then
    timeout -k 10 900 python -u -m pytest $TESTS -m gpu -q -x --timeout 120 --timeout-method thread -rf > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
    tail -2 "$OUT/gpu_tests.log"
fi
IFS='|' read -ra VS <<< "${VARIANTS:-X=0}"
IFS=';' read -ra GS <<< "${GEOS:-1920 1080 8 8}"
for r in $(seq "$ROUNDS"); do
    for geo in "${GS[@]}"; do
        for v in "${VS[@]}"; do
            line=$(env $v timeout -k 10 120 python3 scripts/quick_perf.py $geo 2>/dev/null)
            echo "{\"variant\": \"$v\", \"r\": $line}" >> "$OUT/ab.jsonl"
        done
    done
done
python3 - "$OUT/ab.jsonl" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    j = json.loads(line); r = j["r"]
    d[(r["W"], r["H"], r["spp"], r["env"], j["variant"])].append(r["ms_per_launch"])
for k in sorted(d):
    print(k, ["%.4f" % x for x in d[k]])
PY
