#!/usr/bin/env bash
# Round 4 dev tool: v4 continuous-tiles kernel vs the per-tile one: work counts + timing
# (scripts/v4_perf.py), then SQ counters of both (rocprofv3 --pmc, one pass each).
set -euo pipefail
TAG=${1:-v4ct}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp PT_QP_K=20
for v in ct old; do
  if [ $v = old ]; then export PT_MI355_NO_CT=1; else unset PT_MI355_NO_CT; fi
  timeout -k 10 120 python3 scripts/v4_perf.py > "$OUT/perf_$v.json"
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH --output-format csv -d "$OUT/$v" -o run -- python3 "$PWD/scripts/v4_perf.py" > "$OUT/$v.log" 2>&1
done
cat "$OUT"/perf_*.json
python3 - "$OUT" <<'PY'
import collections, csv, glob, sys
for v in ("ct", "old"):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"{sys.argv[1]}/{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "v4" in k and "ELb0ELb1ELi1ELb1E" in r["Kernel_Name"].replace("<", "").replace(">", "") or ("v4" in k and "false, true, 1, true" in k):
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(v, {k: "%.4g" % (sum(x) / len(x)) for k, x in sorted(agg.items())})
PY
