#!/usr/bin/env bash
# Round 4 dev tool: per-wave / per-tile timelines (diagnostic build, scripts/diag_timeline.py) of the
# continuous-tiles pool and of render_body (PT_MI355_NO_CT=1), for geometries "W H S B" ...
set -euo pipefail
TAG=$1; shift
OUT=gpurun_out/diag/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp PT_MI355_LIB=build/libpt_diag.so
for geo in "$@"; do
    n=$(echo $geo | tr ' ' _)
    PT_DIAG_FILE=$OUT/ct_$n.bin timeout -k 10 120 python3 scripts/diag_timeline.py $geo > "$OUT/ct_$n.json" 2> "$OUT/ct_$n.err"
    PT_MI355_NO_CT=1 PT_DIAG_FILE=$OUT/old_$n.bin timeout -k 10 120 python3 scripts/diag_timeline.py $geo > "$OUT/old_$n.json" 2> "$OUT/old_$n.err"
    rm -f "$OUT"/*.bin
    echo "== $geo"; cat "$OUT/ct_$n.json" "$OUT/old_$n.json"
done
