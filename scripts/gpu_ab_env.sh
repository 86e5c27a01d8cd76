# Dev tool: GPU suite, then interleaved c4 / v4 timings of the working tree against build/libpt_$BASE.so
#   bash scripts/gpu_ab_env.sh TAG BASE
set -euo pipefail
export TMPDIR=/tmp
TAG=$1; BASE=$2
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
export PT_QP_K=60
for r in 1 2 3; do
  bash scripts/ab.sh $OUT/ab_c4.jsonl "1920 1080 16 8 env" default build/libpt_$BASE.so
  bash scripts/ab_v4.sh $OUT/ab_v4.jsonl "1920 1080 8 8 equirect" default build/libpt_$BASE.so
done
python3 - $OUT <<'PY'
import json, sys, collections, glob
for f in sorted(glob.glob(f"{sys.argv[1]}/ab_*.jsonl")):
    d = collections.defaultdict(list)
    for line in open(f):
        j = json.loads(line); d[j["lib"].split("/")[-1]].append(j["ms_per_launch"])
    print(f.split("/")[-1], {k: ["%.4f" % x for x in v] for k, v in d.items()})
PY
