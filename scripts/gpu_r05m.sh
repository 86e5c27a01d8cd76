#!/usr/bin/env bash
# Round 5: the env kernel's timed back-claim arms (pt_capi.cpp ct_occupancy): the env / output / regime
# parity tests, then the c4 bench interleaved -- default (timed arms) against PT_MI355_BACK=20 (the
# previous fixed share; a given PT_MI355_BACK turns the env arms off).
set -euo pipefail
TAG=${1:-r05m}; OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_env.py tests/test_gpu_regime.py tests/test_gpu_output.py > "$OUT/tests.log" 2>&1
tail -3 "$OUT/tests.log"
for r in 1 2 3; do
  for v in "X=0" "PT_MI355_BACK=20"; do
    env $v timeout -k 10 200 python3 bench.py --workload c4_env_1080p --no-cpu-baseline > "$OUT/c4.json" 2>/dev/null
    echo "{\"variant\": \"$v\", \"wl\": \"c4\", \"ms\": $(python3 -c "import json;print(json.loads(open('$OUT/c4.json').read().strip().splitlines()[-1])['ms_per_step'])")}" >> "$OUT/bench_ab.jsonl"
  done
done
cat "$OUT/bench_ab.jsonl"
