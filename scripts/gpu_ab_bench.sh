#!/usr/bin/env bash
# Dev tool: interleaved A/B of library settings on bench.py workloads (kernel-inclusive ms/step).
#   VARIANTS="A=1|A=0" WORKLOADS="v4_1080p c2_1080p" bash scripts/gpu_ab_bench.sh TAG ROUNDS
# TESTS="pytest args" runs those -m gpu tests first.  Output: gpurun_out/TAG/ab_bench.jsonl + summary.
set -euo pipefail
TAG=${1:-abb}; ROUNDS=${2:-2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
    timeout -k 10 900 python -u -m pytest $TESTS -m gpu -q -x --timeout 120 --timeout-method thread -rf > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
    tail -2 "$OUT/gpu_tests.log"
fi
IFS='|' read -ra VS <<< "${VARIANTS:-X=0}"
for r in $(seq "$ROUNDS"); do
    for wl in ${WORKLOADS:-v4_1080p}; do
        for v in "${VS[@]}"; do
            line=$(env $v timeout -k 10 180 python3 bench.py --workload "$wl" --steps ${STEPS:-40} --warmup 5 --no-cpu-baseline 2>/dev/null | grep '^{')
            echo "{\"variant\": \"$v\", \"workload\": \"$wl\", \"r\": $line}" >> "$OUT/ab_bench.jsonl"
        done
    done
done
python3 - "$OUT/ab_bench.jsonl" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    j = json.loads(line)
    d[(j["workload"], j["variant"])].append(j["r"]["ms_per_step"])
for k in sorted(d):
    print(k, ["%.4f" % x for x in d[k]])
PY
