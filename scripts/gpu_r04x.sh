#!/usr/bin/env bash
# Round 4 (x): the bench line of every workload after the r04z profiles were summarised (bench.py
# reads the committed pmc_summary files for its roofline `traffic`), for profiles/r04z_bench_*.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04x
mkdir -p $OUT
timeout -k 10 300 python3 bench.py > $OUT/bench_c2_1080p.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
for wl in c3_4k c4_env_1080p v4_1080p c5_8k; do
    timeout -k 10 300 python3 bench.py --workload $wl --no-cpu-baseline > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || { tail -20 $OUT/bench_$wl.err; exit 1; }
done
for f in $OUT/bench_*.json; do python3 -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f',d['ms_per_step'],'%.3e'%d['value'],d['roofline']['frac'],d['roofline'].get('traffic'))"; done
