# Dev tool: the ring pool against the chunked pool by frame count (gpurun)
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03y
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf -x > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
for r in 1 2; do
  for s in 16 24 32 48; do PT_QP_K=40 bash scripts/ab.sh $OUT/ab_1080p_$s.jsonl "1920 1080 $s 8" build/libpt_ringall.so build/libpt_ringnone.so; done
  PT_QP_K=4 bash scripts/ab.sh $OUT/ab_c5.jsonl "7680 4320 256 8" build/libpt_ringall.so build/libpt_ringnone.so
done
python3 - $OUT <<'PY'
import json, sys, collections, glob
for f in sorted(glob.glob(f"{sys.argv[1]}/ab_*.jsonl")):
    d = collections.defaultdict(list)
    for line in open(f):
        j = json.loads(line); d[j["lib"].split("/")[-1]].append(j["ms_per_launch"])
    print(f.split("/")[-1], {k: ["%.4f" % x for x in v] for k, v in d.items()})
PY
