# Dev tool: interleaved timings of the working tree's library and build/ variants (gpurun):
#   bash scripts/gpu_timing.sh TAG v4|diffuse "W H S B [mode]" VARIANT...
set -euo pipefail
export TMPDIR=/tmp PT_QP_K=60
OUT=gpurun_out/$1; KIND=$2; ARGS=$3; shift 3
mkdir -p $OUT
libs=(default)
for v in "$@"; do libs+=(build/libpt_$v.so); done
runner=scripts/ab.sh
[ "$KIND" = v4 ] && runner=scripts/ab_v4.sh
for r in 1 2 3; do bash $runner $OUT/ab_$KIND.jsonl "$ARGS" "${libs[@]}"; done
python3 - $OUT <<'PY'
import json, sys, collections, glob
for f in sorted(glob.glob(f"{sys.argv[1]}/ab_*.jsonl")):
    d = collections.defaultdict(list)
    for line in open(f):
        j = json.loads(line); d[j["lib"].split("/")[-1]].append(j["ms_per_launch"])
    print(f.split("/")[-1], {k: ["%.4f" % x for x in v] for k, v in d.items()})
PY
