# Dev tool: parity + timing of ring-pool variants (gpurun)
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03r2
mkdir -p $OUT
for v in rpm8 rpm; do
  PT_MI355_LIB=$PWD/build/libpt_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q --timeout 120 --timeout-method thread -rf -x > $OUT/tests_$v.log 2>&1 || { tail -30 $OUT/tests_$v.log; exit 1; }
  tail -1 $OUT/tests_$v.log
done
for r in 1 2; do
  PT_QP_K=60 bash scripts/ab.sh $OUT/ab_c2.jsonl "1920 1080 8 8" default build/libpt_r8.so build/libpt_rpm8.so
  PT_QP_K=40 bash scripts/ab.sh $OUT/ab_1080p16.jsonl "1920 1080 16 8" default build/libpt_r8.so build/libpt_rpm8.so
  PT_QP_K=10 bash scripts/ab.sh $OUT/ab_c3.jsonl "3840 2160 64 8" default build/libpt_rpm.so
  PT_QP_K=4 bash scripts/ab.sh $OUT/ab_c5.jsonl "7680 4320 256 8" default build/libpt_rpm.so
done
python3 - $OUT <<'PY'
import json, sys, collections, glob
for f in sorted(glob.glob(f"{sys.argv[1]}/ab_*.jsonl")):
    d = collections.defaultdict(list)
    for line in open(f):
        j = json.loads(line); d[j["lib"].split("/")[-1]].append(j["ms_per_launch"])
    print(f.split("/")[-1], {k: ["%.4f" % x for x in v] for k, v in d.items()})
PY
