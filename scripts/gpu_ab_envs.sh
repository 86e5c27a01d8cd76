#!/usr/bin/env bash
# A/B of environment switches on the default bench line (dev tool), interleaved ROUNDS times:
#   bash scripts/gpu_ab_envs.sh TAG ROUNDS WORKLOAD "ENV=1 ENV2=x" "ENV=2" ...   ("-" : no switch)
# each variant runs bench.py (chained steps unless the variant says --no-chain via NOCHAIN=1)
set -uo pipefail
TAG=$1; R=$2; WL=$3; shift 3
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
for r in $(seq "$R"); do
    i=0
    for v in "$@"; do
        i=$((i + 1))
        extra=()
        [ "$v" = "-" ] && v=""
        case " $v " in *" NOCHAIN=1 "*) extra=(--no-chain) ;; esac
        env $v timeout -k 10 200 python3 bench.py --workload "$WL" --steps 200 --no-cpu-baseline --no-configs4 "${extra[@]}" \
            > "$OUT/v${i}_$r.json" 2> "$OUT/v${i}_$r.err" || { tail -5 "$OUT/v${i}_$r.err"; exit 1; }
        python3 -c "import json;d=json.loads(open('$OUT/v${i}_$r.json').read().strip().splitlines()[-1]);print('[$v]', $r, round(d['ms_per_step'], 5), round(d['roofline']['frac'], 4), d.get('launch_variant'), {k: v for k, v in d.get('launch_chain', {}).items() if k != 'note'})" | tee -a "$OUT/summary.txt"
    done
done
