set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03x
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf -x > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
export PT_QP_K=10
for r in 1 2 3; do
  bash scripts/ab.sh $OUT/ab_c3.jsonl "3840 2160 64 8" default build/libpt_h3.so
  PT_QP_K=60 bash scripts/ab.sh $OUT/ab_1080p16.jsonl "1920 1080 16 8" default build/libpt_h3.so
  PT_QP_K=60 bash scripts/ab.sh $OUT/ab_c2.jsonl "1920 1080 8 8" default build/libpt_h3.so
done
python3 - $OUT <<'PY'
import json, sys, collections, glob
for f in sorted(glob.glob(f"{sys.argv[1]}/ab_*.jsonl")):
    d = collections.defaultdict(list)
    for line in open(f):
        j = json.loads(line); d[j["lib"].split("/")[-1]].append(j["ms_per_launch"])
    print(f.split("/")[-1], {k: ["%.4f" % x for x in v] for k, v in d.items()})
PY
