#!/usr/bin/env bash
# Round-3 GPU call: tests + benches + profiles (gpu_r03d.sh), then interleaved A/B rounds of the
# kernel variants under build/ (diffuse: HEAD kernel, old cull; v4: forced 5 waves).
set -euo pipefail
TAG=${1:-r03e}
bash scripts/gpu_r03d.sh "$TAG"
OUT=gpurun_out/$TAG
export PT_QP_K=60
for r in 1 2 3; do
    bash scripts/ab.sh "$OUT/ab_c2.jsonl" "1920 1080 8 8" default build/libpt_head.so build/libpt_oldcull.so
    bash scripts/ab.sh "$OUT/ab_c3_8spp.jsonl" "3840 2160 8 8" default build/libpt_head.so build/libpt_oldcull.so
    bash scripts/ab_v4.sh "$OUT/ab_v4.jsonl" "1920 1080 8 8 equirect" default build/libpt_v4w5.so
done
python3 - "$OUT" <<'PY'
import json, sys, collections
for f in ("ab_c2.jsonl", "ab_c3_8spp.jsonl", "ab_v4.jsonl"):
    d = collections.defaultdict(list)
    for line in open(f"{sys.argv[1]}/{f}"):
        j = json.loads(line); d[j["lib"].split("/")[-1]].append(j["ms_per_launch"])
    print(f, {k: ["%.4f" % x for x in v] for k, v in d.items()})
PY
