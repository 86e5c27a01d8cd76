#!/usr/bin/env bash
# Round 5: the bench itself (sustained launches, its own warm-up) for the multi-chunk workloads under
# each occupancy, interleaved: c3 / c5 at the default (timed; 6 waves until the pick), 5 and 6 waves
# fixed; c4 with the 6-wave env kernel against the 5-wave build.
set -euo pipefail
TAG=${1:-r05l}; OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 1 2; do
  for v in "X=0" "PT_MI355_CT_WAVES=5" "PT_MI355_CT_WAVES=6"; do
    env $v timeout -k 10 200 python3 bench.py --workload c3_4k --no-cpu-baseline --steps 60 > "$OUT/c3.json" 2>/dev/null
    echo "{\"variant\": \"$v\", \"wl\": \"c3\", \"ms\": $(python3 -c "import json;print(json.loads(open('$OUT/c3.json').read().strip().splitlines()[-1])['ms_per_step'])")}" >> "$OUT/bench_ab.jsonl"
    env $v timeout -k 10 200 python3 bench.py --workload c5_8k --no-cpu-baseline --steps 4 > "$OUT/c5.json" 2>/dev/null
    echo "{\"variant\": \"$v\", \"wl\": \"c5\", \"ms\": $(python3 -c "import json;print(json.loads(open('$OUT/c5.json').read().strip().splitlines()[-1])['ms_per_step'])")}" >> "$OUT/bench_ab.jsonl"
  done
  for v in "X=0" "PT_MI355_LIB=build/libpt_env5.so"; do
    env $v timeout -k 10 200 python3 bench.py --workload c4_env_1080p --no-cpu-baseline > "$OUT/c4.json" 2>/dev/null
    echo "{\"variant\": \"$v\", \"wl\": \"c4\", \"ms\": $(python3 -c "import json;print(json.loads(open('$OUT/c4.json').read().strip().splitlines()[-1])['ms_per_step'])")}" >> "$OUT/bench_ab.jsonl"
  done
done
cat "$OUT/bench_ab.jsonl"
