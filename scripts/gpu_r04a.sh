#!/usr/bin/env bash
# Round 4 (a): the -m gpu suite, then `python bench.py --gpus 2` through bench.spawn_ranks (rehearsal:
# both ranks on the one GPU, gloo) and the default N = 1 bench line.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04a
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
PT_BENCH_REHEARSE=1 timeout -k 10 300 python3 bench.py --gpus 2 --no-cpu-baseline > $OUT/rehearse_n2.json 2> $OUT/rehearse_n2.err || { tail -20 $OUT/rehearse_n2.err; exit 1; }
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/bench_c2.json').read().strip().splitlines()[-1]);print(d['ms_per_step'],d['value'],d['roofline']['frac'])"
