#!/usr/bin/env bash
# Round 4 dev tool: SQ instruction counters of the one-chunk render kernel with and without the
# continuous-tiles pool (PT_MI355_NO_CT), for a geometry: bash scripts/gpu_pmc_ct.sh TAG W H S B
set -euo pipefail
TAG=$1; shift
OUT=$PWD/gpurun_out/pmc/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp PT_QP_K=10
CMD=(python3 "$PWD/scripts/quick_perf.py" "$@")
for v in ct old; do
  if [ $v = old ]; then export PT_MI355_NO_CT=1; else unset PT_MI355_NO_CT; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH --output-format csv -d "$OUT/$v" -o run -- "${CMD[@]}" > "$OUT/$v.log" 2>&1
  timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU_TRANS_F32 --output-format csv -d "$OUT/${v}2" -o run -- "${CMD[@]}" > "$OUT/${v}2.log" 2>&1 || true
done
python3 - "$OUT" <<'PY'
import collections, csv, glob, sys
for v in ("ct", "old"):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"{sys.argv[1]}/{v}*/**/*counter_collection.csv", recursive=True):
        if f"/{v}2/" in f and v == "old" and False: pass
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if ("pt_render_ct_kernel<0, false>" in k) or ("pt_render_kernel<0, false, false, false>" in k):
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(v, {k: "%.4g" % (sum(x) / len(x)) for k, x in sorted(agg.items())})
PY
