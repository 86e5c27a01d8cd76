#!/usr/bin/env bash
# Round 5: the presenting continuous-tiles kernels against the plain ones over the whole image
# (scripts/debug_present.py): every occupancy, c2 geometry, 3 and 10 launches.
set -euo pipefail
TAG=${1:-r05t}; OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in "PT_MI355_CT_WAVES=6" "PT_MI355_CT_WAVES=5" "X=0" "PT_DBG_LAUNCHES=10"; do
  env $v timeout -k 10 300 python3 scripts/debug_present.py >> "$OUT/dbg.jsonl" 2> "$OUT/dbg.err"
done
cat "$OUT/dbg.jsonl"
