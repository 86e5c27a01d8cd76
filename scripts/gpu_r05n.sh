#!/usr/bin/env bash
# Round 5: the fused OutputToScreen of the v4 drop-in (DemofoxRenderOptV4 with screen pixels: the
# per-tile kernel's presenting instance) -- the v4 / output parity tests, the shipping host's frame
# cadence against the previous library (separate tonemap pass), and the c2 bench's fused-present
# measurement with the presenting CT kernel at the launch's occupancy.
set -euo pipefail
TAG=${1:-r05n}; OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_v4.py tests/test_gpu_output.py > "$OUT/tests.log" 2>&1
tail -3 "$OUT/tests.log"
for r in 1 2; do
  for v in "X=0" "PT_MI355_LIB=build/libpt_prev.so"; do
    echo "{\"variant\": \"$v\", \"r\": $(env $v timeout -k 10 200 python3 scripts/host_path_perf_v4.py 1920 1080)}" >> "$OUT/host_v4.jsonl"
  done
done
cat "$OUT/host_v4.jsonl"
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-configs4 > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err"
python3 -c "import json;d=json.loads(open('$OUT/bench_c2.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], json.dumps(d['output_stage']))"
