#!/usr/bin/env bash
# Round 4 (w): c5 (7680x4320, 256 spp, one GPU) -- rocprofv3 trace + PMC passes, summarised on the box,
# then its bench line with that summary (copied back under gpurun_out/r04w).
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04w
mkdir -p $OUT
STEPS=4 bash scripts/round_profile.sh r04z c5_8k
python3 scripts/summarize_profile.py r04z_c5 c5_8k > $OUT/summarize.log
cp profiles/r04z_c5_pmc.txt profiles/r04z_c5_kernel_stats.csv profiles/pmc_summary_c5_8k.json $OUT/
timeout -k 10 300 python3 bench.py --workload c5_8k --no-cpu-baseline > $OUT/bench_c5_8k.json 2> $OUT/bench_c5.err || { tail -20 $OUT/bench_c5.err; exit 1; }
tail -1 $OUT/bench_c5_8k.json
