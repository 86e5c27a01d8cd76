set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03sg
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_v4.py tests/test_gpu_queue.py tests/test_gpu_flags.py tests/test_gpu_multidev.py -m gpu -q --timeout 120 --timeout-method thread -rf > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
export PT_QP_K=60
for r in 1 2 3; do bash scripts/ab_v4.sh $OUT/ab_v4.jsonl "1920 1080 8 8 equirect" default build/libpt_h4.so; done
python3 - $OUT <<'PY'
import json, sys, collections, glob
for f in sorted(glob.glob(f"{sys.argv[1]}/ab_*.jsonl")):
    d = collections.defaultdict(list)
    for line in open(f):
        j = json.loads(line); d[j["lib"].split("/")[-1]].append(j["ms_per_launch"])
    print(f.split("/")[-1], {k: ["%.4f" % x for x in v] for k, v in d.items()})
PY
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $PWD/$OUT/pmc -o run -- python3 scripts/quick_perf_v4.py 1920 1080 8 8 equirect > $OUT/pmc.log 2>&1 || echo "pmc failed"
