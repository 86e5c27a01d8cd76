#!/usr/bin/env bash
# Round 4 (v): the final tree after the occupancy timing -- the -m gpu suite, smoke() and the
# `bench.py --gpus 2` rehearsal through spawn_ranks.
set -euo pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04t}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
PT_BENCH_REHEARSE=1 timeout -k 10 300 python3 bench.py --gpus 2 --no-cpu-baseline > $OUT/rehearse_c2_n2.json 2> $OUT/rehearse_n2.err || { tail -20 $OUT/rehearse_n2.err; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/rehearse_c2_n2.json').read().strip().splitlines()[-1]);print('n2',d['ms_per_step'],'%.3e'%d['value'])"
