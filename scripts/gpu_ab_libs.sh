#!/usr/bin/env bash
# A/B of library variants on the default bench line (dev tool), interleaved ROUNDS times:
#   bash scripts/gpu_ab_libs.sh TAG ROUNDS WORKLOAD VARIANT...
# VARIANT: default | chain (this tree, chained steps) | build/libpt_X.so (plain steps, --no-chain)
set -uo pipefail
TAG=$1; R=$2; WL=$3; shift 3
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
B=(python3 bench.py --workload "$WL" --steps 200 --no-cpu-baseline --no-configs4)
for r in $(seq "$R"); do
    for v in "$@"; do
        n=$(basename "$v" .so)
        case $v in
            default) env -u PT_MI355_LIB timeout -k 10 200 "${B[@]}" --no-chain > "$OUT/${n}_$r.json" 2> "$OUT/${n}_$r.err" ;;
            chain) env -u PT_MI355_LIB timeout -k 10 200 "${B[@]}" > "$OUT/${n}_$r.json" 2> "$OUT/${n}_$r.err" ;;
            *) PT_MI355_LIB=$PWD/$v timeout -k 10 200 "${B[@]}" --no-chain > "$OUT/${n}_$r.json" 2> "$OUT/${n}_$r.err" ;;
        esac || { tail -5 "$OUT/${n}_$r.err"; exit 1; }
        python3 -c "import json;d=json.loads(open('$OUT/${n}_$r.json').read().strip().splitlines()[-1]);print('$n', $r, round(d['ms_per_step'], 5), round(d['roofline']['frac'], 4))" | tee -a "$OUT/summary.txt"
    done
done
