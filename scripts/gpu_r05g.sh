#!/usr/bin/env bash
# Round 5: the v4 continuous-tiles kernel at 6 waves per SIMD (80 VGPRs, 16 KiB LDS per block) against
# its 5-wave build and the per-tile kernel (the default at 1080p 8 spp).
set -euo pipefail
TAG=${1:-r05g}; OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp PT_QP_K=30
for r in 1 2; do
  for geo in "1920 1080 8 8" "3840 2160 8 8" "1920 1080 32 8"; do
    for v in "X=0" "PT_MI355_V4_CT=1" "PT_MI355_V4_CT=1 PT_MI355_LIB=build/libpt_v4w6.so"; do
      line=$(env $v timeout -k 10 120 python3 scripts/v4_perf.py $geo)
      echo "{\"variant\": \"$v\", \"r\": $line}" >> "$OUT/ab.jsonl"
    done
  done
done
python3 - "$OUT/ab.jsonl" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    j = json.loads(line); r = j["r"]
    d[(r["W"], r["H"], r["spp"], j["variant"])].append("%.4f" % r["ms_per_launch"])
for k in sorted(d):
    print(k, d[k])
PY
