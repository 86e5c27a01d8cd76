#!/usr/bin/env bash
# Round 4: the -m gpu suite with the continuous-tiles pool (render_body_ct), then interleaved A/B of
# one-chunk launches against render_body (PT_MI355_NO_CT=1): gpurun_out/TAG/{gpu_tests.log,ab_ct.jsonl}
set -euo pipefail
TAG=${1:-ct}; ROUNDS=${2:-3}; TESTS=${TESTS:-1}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$TESTS" = 1 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
fi
export PT_QP_K=60
for r in $(seq "$ROUNDS"); do
    for geo in "1920 1080 8 8" "3840 2160 8 8" "1920 1080 16 8" "3840 2160 64 8" "1920 1080 1 8"; do
        timeout -k 10 120 python3 scripts/quick_perf.py $geo >> "$OUT/ab_ct.jsonl"
        PT_MI355_NO_CT=1 timeout -k 10 120 python3 scripts/quick_perf.py $geo >> "$OUT/ab_ct.jsonl"
    done
done
python3 - "$OUT/ab_ct.jsonl" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    j = json.loads(line)
    d[(j["W"], j["H"], j["spp"], j["ct"])].append((j["ms_per_launch"], j["simd_eff"]))
for k in sorted(d):
    print(k, ["%.4f/%.3f" % x for x in d[k]])
PY
