#!/usr/bin/env bash
# Round 5: the v4 CT kernel's resolve lambda forced inline (the non-default-flag equirect instances
# called it out of line): v4 parity tests, then 1080p 8 spp v4 launches with bilinear texel sampling
# (PT_QP_RJ=0, a non-default-flag instance) and with the defaults, new vs previous library.
set -euo pipefail
TAG=${1:-r05o}; OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_v4.py > "$OUT/tests.log" 2>&1
tail -3 "$OUT/tests.log"
for r in 1 2; do
  for rj in 0 1; do
    for v in "X=0" "PT_MI355_LIB=build/libpt_prev.so"; do
      echo "{\"variant\": \"$v\", \"rj\": $rj, \"r\": $(env $v PT_QP_RJ=$rj PT_QP_K=100 timeout -k 10 120 python3 scripts/v4_perf.py)}" >> "$OUT/v4_ab.jsonl"
    done
  done
done
python3 -c "
import json
for l in open('$OUT/v4_ab.jsonl'):
    d = json.loads(l); print(d['variant'], d['rj'], round(d['r']['ms_per_launch'], 4))"
