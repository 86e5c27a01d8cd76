#!/usr/bin/env bash
# A/B of the default bench line (dev tool): the pre-chain library (PT_MI355_LIB=build/libpt_prechain.so,
# plain launches), this tree plain (--no-chain) and this tree chained, interleaved ROUNDS times.
#   bash scripts/gpu_ab_chain.sh TAG [ROUNDS] [WORKLOAD]
set -uo pipefail
TAG=$1; R=${2:-2}; WL=${3:-c2_1080p}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
B=(python3 bench.py --workload "$WL" --steps 200 --no-cpu-baseline --no-configs4)
for r in $(seq "$R"); do
    PT_MI355_LIB=$PWD/build/libpt_prechain.so timeout -k 10 200 "${B[@]}" --no-chain > "$OUT/pre_$r.json" 2> "$OUT/pre_$r.err" || exit 1
    timeout -k 10 200 "${B[@]}" --no-chain > "$OUT/plain_$r.json" 2> "$OUT/plain_$r.err" || exit 1
    timeout -k 10 200 "${B[@]}" > "$OUT/chain_$r.json" 2> "$OUT/chain_$r.err" || exit 1
    for v in pre plain chain; do
        python3 -c "import json;d=json.loads(open('$OUT/${v}_$r.json').read().strip().splitlines()[-1]);print('$v', $r, round(d['ms_per_step'], 5), round(d['roofline']['frac'], 4))"
    done
done
