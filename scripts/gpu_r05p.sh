#!/usr/bin/env bash
# Round 5: per-wave birth / death of one c2 launch (diagnostic build, waves only) under the default
# timed variants and the fixed ones: how much of the launch's end is idle now.
set -euo pipefail
TAG=${1:-r05p}; OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp PT_MI355_LIB=build/libpt_diag.so
for v in "X=0" "PT_MI355_CT_WAVES=6 PT_MI355_BACK=45" "PT_MI355_CT_WAVES=6" "PT_MI355_CT_WAVES=5"; do
  for geo in "1920 1080 8 8" "3840 2160 8 8"; do
    echo "{\"variant\": \"$v\", \"geo\": \"$geo\", \"r\": $(env $v PT_DIAG_FILE=$OUT/d.bin timeout -k 10 120 python3 scripts/diag_timeline.py $geo)}" >> "$OUT/diag.jsonl"
    rm -f "$OUT/d.bin"
  done
done
python3 -c "
import json
for l in open('$OUT/diag.jsonl'):
    d = json.loads(l); r = d['r']; print(d['variant'], d['geo'], r['span_us'], r['idle_frac_end'], r['death_us_pct'])"
