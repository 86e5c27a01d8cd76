#!/usr/bin/env bash
# A/B timing of v4 library variants on the GPU box (dev tool):
#   bash scripts/ab_v4.sh OUT.jsonl "W H S B mode" default build/libpt_x.so ...
set -euo pipefail
OUT=$1; ARGS=$2; shift 2
mkdir -p "$(dirname "$OUT")"
for v in "$@"; do
    if [ "$v" = default ]; then unset PT_MI355_LIB; else export PT_MI355_LIB=$PWD/$v; fi
    timeout -k 10 120 python3 scripts/quick_perf_v4.py $ARGS >> "$OUT" 2>/dev/null
done
