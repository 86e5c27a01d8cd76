#!/usr/bin/env bash
# GPU tests + benches, then interleaved A/B of the working tree against build/libpt_$BASE.so.
set -euo pipefail
TAG=${1:-r03h}; BASE=${2:-c0f}
OUT=gpurun_out/$TAG
bash scripts/gpu_r03c.sh "$TAG"
export PT_QP_K=60
for r in 1 2 3; do
    bash scripts/ab.sh "$OUT/ab_c2.jsonl" "1920 1080 8 8" default build/libpt_$BASE.so
    bash scripts/ab.sh "$OUT/ab_c3_8spp.jsonl" "3840 2160 8 8" default build/libpt_$BASE.so
    bash scripts/ab.sh "$OUT/ab_c4.jsonl" "1920 1080 16 8 env" default build/libpt_$BASE.so
done
python3 - "$OUT" <<'PY'
import json, sys, collections
for f in ("ab_c2.jsonl", "ab_c3_8spp.jsonl", "ab_c4.jsonl"):
    d = collections.defaultdict(list)
    for line in open(f"{sys.argv[1]}/{f}"):
        j = json.loads(line); d[j["lib"].split("/")[-1]].append(j["ms_per_launch"])
    print(f, {k: ["%.4f" % x for x in v] for k, v in d.items()})
PY
