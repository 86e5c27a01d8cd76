#!/usr/bin/env bash
# Round 4 (u): after the occupancy timing -- the c5 profile (summarised on the box: its traces are
# large) and the bench lines of c4 / v4 (kernels unchanged) and c5, for profiles/r04t_*.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04t
mkdir -p $OUT
STEPS=4 bash scripts/round_profile.sh r04t c5_8k
python3 scripts/summarize_profile.py r04t_c5 c5_8k > $OUT/summarize_c5.log
cp profiles/r04t_c5_pmc.txt profiles/r04t_c5_kernel_stats.csv profiles/pmc_summary_c5_8k.json $OUT/
rm -rf gpurun_out/prof/r04t_c5
for wl in c4_env_1080p v4_1080p c5_8k; do
    timeout -k 10 300 python3 bench.py --workload $wl --no-cpu-baseline > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || { tail -20 $OUT/bench_$wl.err; exit 1; }
done
for f in $OUT/bench_*.json; do python3 -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f',d['ms_per_step'],'%.3e'%d['value'],d['roofline']['frac'])"; done
