#!/usr/bin/env bash
# Round 5: the v4 continuous-tiles kernel (default-flags instance) at 7 waves per SIMD
# (build/libpt_v4w7.so, -DPT_V4_CT_DFL_WAVES=7: 72 VGPRs, no scratch in its pool loop) against 6,
# interleaved: the v4 bench workload (1080p 8 spp), 1080p 32 spp, 4K 8 spp.
set -euo pipefail
TAG=${1:-r05y}; OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
PT_MI355_LIB=build/libpt_v4w7.so timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_v4.py > "$OUT/tests.log" 2>&1
tail -1 "$OUT/tests.log"
for r in 1 2 3; do
  for geo in "1920 1080 8 8" "1920 1080 32 8" "3840 2160 8 8"; do
    for v in "X=0" "PT_MI355_LIB=build/libpt_v4w7.so"; do
      echo "{\"variant\": \"$v\", \"geo\": \"$geo\", \"r\": $(env $v PT_QP_K=60 timeout -k 10 120 python3 scripts/v4_perf.py $geo)}" >> "$OUT/ab.jsonl"
    done
  done
done
python3 -c "
import json, collections
d = collections.defaultdict(list)
for l in open('$OUT/ab.jsonl'):
    x = json.loads(l); d[(x['geo'], x['variant'])].append(x['r']['ms_per_launch'])
for k in sorted(d): print(k, [round(v, 4) for v in d[k]], round(sum(d[k]) / len(d[k]), 4))"
