#!/usr/bin/env bash
# Chained launches on the GPU: the chain tests, then the default bench line with and without chaining.
# usage: scripts/gpu_chain_check.sh TAG [pytest -k expression]
set -uo pipefail
TAG=${1:-chain}; OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
(while sleep 45; do date >> "$OUT/heartbeat"; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
K=${2:-}
timeout -k 10 800 python -u -m pytest tests/test_gpu_chain.py -x -v --timeout 400 --timeout-method thread --durations=0 \
    ${K:+-k "$K"} > "$OUT/chain_tests.log" 2>&1 || { tail -40 "$OUT/chain_tests.log"; exit 1; }
tail -15 "$OUT/chain_tests.log"
WL=${WORKLOADS:-c2_1080p}
for wl in $WL; do
    timeout -k 10 200 python bench.py --workload "$wl" --no-cpu-baseline --no-configs4 > "$OUT/bench_chain_$wl.json" 2> "$OUT/bench_chain_$wl.err" || { tail -20 "$OUT/bench_chain_$wl.err"; exit 1; }
    timeout -k 10 200 python bench.py --workload "$wl" --no-cpu-baseline --no-configs4 --no-chain > "$OUT/bench_nochain_$wl.json" 2> "$OUT/bench_nochain_$wl.err" || { tail -20 "$OUT/bench_nochain_$wl.err"; exit 1; }
done
for f in $(for wl in $WL; do echo bench_chain_$wl bench_nochain_$wl; done); do
    python3 -c "import json;d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]);print('$f', d['ms_per_step'], '%.3e' % d['value'], round(d['roofline']['frac'], 4), d.get('launch_chain'))"
done
