#!/usr/bin/env bash
# Every bench workload on the GPU box (run via gpurun from the repo root):
#   bash scripts/gpu_benches.sh TAG  -> gpurun_out/TAG/bench_<workload>.json
# c2 with its CPU baseline (the driver's default line), the others without.
set -euo pipefail
TAG=${1:-bench}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > "$OUT/bench_c2_1080p.json" 2> "$OUT/bench_c2_1080p.err"
for wl in c3_4k c4_env_1080p v4_1080p c5_8k; do
    timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline > "$OUT/bench_$wl.json" 2> "$OUT/bench_$wl.err"
done
python - "$OUT" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(f"{sys.argv[1]}/bench_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], "%.4g" % d["value"], "kernel_ms %.4f" % d["kernel_ms_avg"], "frac %.4f" % d["roofline"]["frac"],
          "cpu", (d.get("cpu_baseline") or {}).get("value"))
PY
