#!/usr/bin/env bash
# Round 4 (t): after the per-geometry occupancy timing of the diffuse CT kernel (5 / 6 waves per
# SIMD) -- rocprofv3 kernel traces + PMC passes of c2 and c3 and their bench lines, for profiles/r04t_*.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04t
mkdir -p $OUT
STEPS=10 bash scripts/round_profile.sh r04t c2_1080p c3_4k
timeout -k 10 300 python3 bench.py > $OUT/bench_c2_1080p.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
timeout -k 10 300 python3 bench.py --workload c3_4k --no-cpu-baseline > $OUT/bench_c3_4k.json 2> $OUT/bench_c3.err || { tail -20 $OUT/bench_c3.err; exit 1; }
for f in $OUT/bench_*.json; do python3 -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f',d['ms_per_step'],'%.3e'%d['value'],d['roofline']['frac'])"; done
