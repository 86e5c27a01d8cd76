#!/usr/bin/env bash
# v4 workload: bench line + rocprofv3 kernel trace (GPU box, from the repo root)
set -euo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload v4_1080p --steps 10 --warmup 2 --cpu-seconds 8 > gpurun_out/bench_v4.json 2> gpurun_out/bench_v4.err
tail -c 3000 gpurun_out/bench_v4.json
TRACE_ONLY=1 WORKLOAD=v4_1080p STEPS=10 bash scripts/profile_gpu.sh "${TAG:-r01e_v4}" > /dev/null
python scripts/summarize_profile.py ${TAG:-r01e_v4} v4_1080p 2>&1 | tail -20 || true
