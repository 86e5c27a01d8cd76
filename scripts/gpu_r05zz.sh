#!/usr/bin/env bash
# Round 5, last: pt_launch_variant (the regime tests) and the bench lines that now report it.
set -euo pipefail
TAG=${1:-r05zz}; OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_regime.py tests/test_gpu_output.py > "$OUT/tests.log" 2>&1
tail -2 "$OUT/tests.log"
timeout -k 10 300 python3 bench.py --no-cpu-baseline > "$OUT/bench_c2_1080p.json" 2> "$OUT/bench_c2.err"
timeout -k 10 300 python3 bench.py --workload c4_env_1080p --no-cpu-baseline > "$OUT/bench_c4_env_1080p.json" 2> "$OUT/bench_c4.err"
for f in "$OUT"/bench_*.json; do python3 -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f', d['ms_per_step'], d.get('launch_variant'))"; done
