#!/usr/bin/env bash
set -euo pipefail
TAG=${1:-r05s}; OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in "PT_MI355_CT_WAVES=6" "PT_MI355_CT_WAVES=5" "X=0"; do
  env $v timeout -k 10 300 python3 scripts/debug_present.py >> "$OUT/dbg.jsonl" 2> "$OUT/dbg.err"
done
cat "$OUT/dbg.jsonl"
