# Dev tool: interleaved v4 timings of the working tree and build/ variants (gpurun):
#   bash scripts/gpu_v4_timing.sh TAG "W H S B mode" VARIANT...
set -euo pipefail
export TMPDIR=/tmp PT_QP_K=60
OUT=gpurun_out/$1; ARGS=$2; shift 2
mkdir -p $OUT
libs=(default)
for v in "$@"; do libs+=(build/libpt_$v.so); done
for r in 1 2 3; do bash scripts/ab_v4.sh $OUT/ab_v4.jsonl "$ARGS" "${libs[@]}"; done
python3 - $OUT <<'PY'
import json, sys, collections, glob
for f in sorted(glob.glob(f"{sys.argv[1]}/ab_*.jsonl")):
    d = collections.defaultdict(list)
    for line in open(f):
        j = json.loads(line); d[j["lib"].split("/")[-1]].append(j["ms_per_launch"])
    print(f.split("/")[-1], {k: ["%.4f" % x for x in v] for k, v in d.items()})
PY
