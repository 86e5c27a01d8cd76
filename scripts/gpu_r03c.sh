#!/usr/bin/env bash
# GPU tests + headline benches after the round-3 boundary / flags / cleanup changes.
set -euo pipefail
TAG=${1:-r03c}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err"
timeout -k 10 300 python bench.py --workload v4_1080p --no-cpu-baseline > "$OUT/bench_v4.json" 2> "$OUT/bench_v4.err"
python - "$OUT" <<'PY'
import json, sys
for f in ("bench_c2.json", "bench_v4.json"):
    d = json.loads(open(f"{sys.argv[1]}/{f}").read().strip().splitlines()[-1])
    print(f, "%.4g" % d["value"], "kernel_ms %.4f" % d["kernel_ms_avg"], "frac %.4f" % d["roofline"]["frac"])
PY
