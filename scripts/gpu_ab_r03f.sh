#!/usr/bin/env bash
# A/B of the v4 kernel across round-2 / HEAD / working-tree builds (dev tool, gpurun).
set -euo pipefail
OUT=gpurun_out/r03f
mkdir -p $OUT
export PT_QP_K=60
for r in 1 2 3; do
    timeout -k 10 120 python3 build/r02/scripts/quick_perf_v4.py 1920 1080 8 8 equirect >> $OUT/ab_v4.jsonl
    bash scripts/ab_v4.sh "$OUT/ab_v4.jsonl" "1920 1080 8 8 equirect" default build/libpt_head.so build/libpt_v4w5.so
    timeout -k 10 120 python3 build/r02/scripts/quick_perf.py 1920 1080 8 8 >> $OUT/ab_c2.jsonl
    bash scripts/ab.sh "$OUT/ab_c2.jsonl" "1920 1080 8 8" default
done
python3 - "$OUT" <<'PY'
import json, sys, collections
for f in ("ab_v4.jsonl", "ab_c2.jsonl"):
    d = collections.defaultdict(list)
    for line in open(f"{sys.argv[1]}/{f}"):
        j = json.loads(line); d[j.get("lib", "r02").split("/")[-1]].append(j["ms_per_launch"])
    print(f, {k: ["%.4f" % x for x in v] for k, v in d.items()})
PY
