# Dev tool: batched ring folds (gpurun)
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03f2
mkdir -p $OUT
for v in r8k4 k4; do
  PT_MI355_LIB=$PWD/build/libpt_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q --timeout 120 --timeout-method thread -rf -x > $OUT/tests_$v.log 2>&1 || { tail -30 $OUT/tests_$v.log; exit 1; }
  tail -1 $OUT/tests_$v.log
done
for r in 1 2; do
  PT_QP_K=60 bash scripts/ab.sh $OUT/ab_c2.jsonl "1920 1080 8 8" default build/libpt_r8k1.so build/libpt_r8k4.so
  PT_QP_K=10 bash scripts/ab.sh $OUT/ab_c3.jsonl "3840 2160 64 8" default build/libpt_k2.so build/libpt_k4.so
  PT_QP_K=4 bash scripts/ab.sh $OUT/ab_c5.jsonl "7680 4320 256 8" default build/libpt_k4.so
done
python3 - $OUT <<'PY'
import json, sys, collections, glob
for f in sorted(glob.glob(f"{sys.argv[1]}/ab_*.jsonl")):
    d = collections.defaultdict(list)
    for line in open(f):
        j = json.loads(line); d[j["lib"].split("/")[-1]].append(j["ms_per_launch"])
    print(f.split("/")[-1], {k: ["%.4f" % x for x in v] for k, v in d.items()})
PY
