#!/usr/bin/env bash
# Round-end check: the tree's whole -m gpu suite, smoke() and the default bench line.
set -euo pipefail
TAG=${1:-round_check}; OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf -p no:cacheprovider > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 300 python3 bench.py > "$OUT/bench_c2_1080p.json" 2> "$OUT/bench_c2.err" || { tail -20 "$OUT/bench_c2.err"; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/bench_c2_1080p.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], '%.3e' % d['value'], d['roofline']['frac'], d.get('launch_variant'))"
