#!/usr/bin/env bash
# Round 4 dev tool: 4-frame continuous-tiles chunks (build/libpt_ch4.so, PT_CT_CHUNK=4) against the
# default 8: timing (scripts/gpu_ab.sh) and the fabric bytes of the c2 kernel (WRITE_SIZE, FETCH_SIZE).
set -euo pipefail
export TMPDIR=/tmp
VARIANTS="X=0|PT_MI355_LIB=build/libpt_ch4.so" GEOS="1920 1080 8 8;1920 1080 16 8 env;3840 2160 64 8" bash scripts/gpu_ab.sh ch4 2
OUT=$PWD/gpurun_out/ch4
for v in def ch4; do
  if [ $v = ch4 ]; then export PT_MI355_LIB=build/libpt_ch4.so; else unset PT_MI355_LIB; fi
  for c in WRITE_SIZE FETCH_SIZE; do
    PT_QP_K=10 timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/${v}_$c" -o run -- python3 "$PWD/scripts/quick_perf.py" > "$OUT/${v}_$c.log" 2>&1
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
for v in ("def", "ch4"):
    for c in ("WRITE_SIZE", "FETCH_SIZE"):
        vals = [float(r["Counter_Value"]) for f in glob.glob(f"{sys.argv[1]}/{v}_{c}/**/*counter_collection.csv", recursive=True)
                for r in csv.DictReader(open(f)) if "pt_render_ct_kernel<0, false>" in r["Kernel_Name"]]
        print(v, c, "%.4g KiB" % (sum(vals) / max(1, len(vals))), len(vals))
PY
