#!/usr/bin/env bash
set -euo pipefail
TAG=${1:-r05r}; OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for k in 8 0; do
  PT_MI355_LATE_SPLIT=$k timeout -k 10 300 python3 scripts/debug_late_split.py >> "$OUT/dbg.jsonl" 2> "$OUT/dbg_$k.err"
done
cat "$OUT/dbg.jsonl"
