#!/usr/bin/env bash
# GPU tests + benches, then v4 A/B against the round-2 build (dev tool, gpurun).
set -euo pipefail
TAG=${1:-r03g}
OUT=gpurun_out/$TAG
bash scripts/gpu_r03c.sh "$TAG"
export PT_QP_K=60
for r in 1 2 3; do
    timeout -k 10 120 python3 build/r02/scripts/quick_perf_v4.py 1920 1080 8 8 equirect | sed 's/"lib": "default"/"lib": "r02"/' >> $OUT/ab_v4.jsonl
    bash scripts/ab_v4.sh "$OUT/ab_v4.jsonl" "1920 1080 8 8 equirect" default
    bash scripts/ab_v4.sh "$OUT/ab_v4_none.jsonl" "1920 1080 8 8 none" default
done
python3 - "$OUT" <<'PY'
import json, sys, collections
for f in ("ab_v4.jsonl", "ab_v4_none.jsonl"):
    d = collections.defaultdict(list)
    for line in open(f"{sys.argv[1]}/{f}"):
        j = json.loads(line); d[j["lib"].split("/")[-1]].append(j["ms_per_launch"])
    print(f, {k: ["%.4f" % x for x in v] for k, v in d.items()})
PY
