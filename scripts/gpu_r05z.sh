#!/usr/bin/env bash
# Round 5 (z): the tree's -m gpu suite, smoke(), `bench.py --gpus 2` rehearsal through spawn_ranks, the
# bench line of every workload (c2 with its CPU baseline and configs[4] leg), and the rocprofv3
# evidence (kernel trace + PMC passes) of every bench workload.
set -euo pipefail
export TMPDIR=/tmp
TAG=${1:-r05z}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
PT_BENCH_REHEARSE=1 timeout -k 10 300 python3 bench.py --gpus 2 --no-cpu-baseline > $OUT/rehearse_c2_n2.json 2> $OUT/rehearse_n2.err || { tail -20 $OUT/rehearse_n2.err; exit 1; }
timeout -k 10 300 python3 bench.py > $OUT/bench_c2_1080p.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
for wl in c3_4k c4_env_1080p v4_1080p c5_8k; do
    timeout -k 10 300 python3 bench.py --workload $wl --no-cpu-baseline > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || { tail -20 $OUT/bench_$wl.err; exit 1; }
done
for f in $OUT/bench_*.json; do python3 -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f',d['ms_per_step'],'%.3e'%d['value'],d['roofline']['frac'])"; done
STEPS=20 bash scripts/round_profile.sh $TAG c2_1080p c3_4k c4_env_1080p v4_1080p > $OUT/profile.log 2>&1 || { tail -20 $OUT/profile.log; exit 1; }
echo profiles done
