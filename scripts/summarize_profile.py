#!/usr/bin/env python3
"""Turn a gpurun_out/prof/<tag> directory (scripts/profile_gpu.sh) into committed summaries:
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (as produced)
  profiles/<tag>_pmc.txt            per-counter means for the render kernel (non-COUNT instance)
  profiles/pmc_summary.json         HBM bytes per launch of the render kernel (read by bench.py);
                                    pmc_summary_<workload>.json for workloads other than c2_1080p
usage: summarize_profile.py TAG [WORKLOAD]

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE from separate passes (KiB).
The guide's x2 correction is for 16-B-per-lane streaming reads; this kernel reads the accumulator
with 12-B-per-lane `global_load_dwordx3` (3 consecutive dwords per pixel).  WRITE_SIZE matches the
known written bytes (W*H*12) to 3 %, and the raw FETCH_SIZE is 0.90x the known read bytes -- a
doubled count would claim 1.8x -- so the raw counters are used, both figures are recorded.
"""
import collections
import csv
import glob
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
tag = sys.argv[1]
workload = sys.argv[2] if len(sys.argv) > 2 else "c2_1080p"
src = ROOT / "gpurun_out" / "prof" / tag
dst = ROOT / "profiles"
dst.mkdir(exist_ok=True)
ENV = workload.startswith("c4")
# Family prefix of the timed (COUNT = false) instance; the remaining template arguments (MULTI for
# launches that chain chunks, v4's exp switch) are resolved below to the instance with the most
# kernel-trace time.
# (round 4: the continuous-tiles kernels, pt_kernel.hip render_body_ct; PT_MI355_NO_CT=1 profiles of the
# per-tile pool: PT_PROFILE_PER_TILE=1)
import os
if os.environ.get("PT_PROFILE_PER_TILE") == "1":
    KERNEL = "pt_render_env_kernel<0, false," if ENV else "pt_render_kernel<0, false,"
else:
    KERNEL = "pt_render_ct_env_kernel<0, false" if ENV else "pt_render_ct_kernel<0, false"
if workload.startswith("v4"):
    # <EQUIRECT, INTERLEAVED, COUNT = false, default-scene literals, FEXP>: the continuous-tiles kernel at
    # the bench's 1080p 8 spp since round 5 (launches of >= 4 chunks per wave), the per-tile one else
    KERNEL = os.environ.get("PT_PROFILE_V4_KERNEL", "pt_v4_ct_kernel<1, 0, false, true,")
SUMMARY = "pmc_summary.json" if workload == "c2_1080p" else f"pmc_summary_{workload}.json"

stats = glob.glob(str(src / "trace" / "**" / "*kernel_stats.csv"), recursive=True)
if stats:
    shutil.copy(stats[0], dst / f"{tag}_kernel_stats.csv")
    rows = [r for r in csv.DictReader(open(stats[0])) if KERNEL in r["Name"]]
    if rows:
        best = max(rows, key=lambda r: float(r["TotalDurationNs"]))["Name"]
        KERNEL = best[best.index(KERNEL):best.index(">", best.index(KERNEL)) + 1]
agg = collections.defaultdict(list)
for f in glob.glob(str(src / "**" / "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if KERNEL in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
mean = {k: sum(v) / len(v) for k, v in agg.items()}
lines = [f"# rocprofv3 PMC means per dispatch of {KERNEL} ({tag})"]
for k in sorted(mean):
    lines.append(f"{k:28s} n={len(agg[k]):3d} mean={mean[k]:.6g}")
avg_ns = None
if stats:
    for r in csv.DictReader(open(stats[0])):
        if KERNEL in r["Name"]:
            avg_ns = float(r["AverageNs"])
            lines.append(f"kernel_trace_average_ns      {avg_ns:.1f} (calls={r['Calls']})")
# The same command's launches after its clock ramp: bench.py's device warm-up runs the first ~25 ms at
# rising clocks (e.g. c2's first 50 launches ~267 us, the steady ones ~240 us), and the
# stats' average includes them.  The per-dispatch trace gives the steady average -- dispatches after
# the first 25 % of the instance's (at least 30 ms of launches), the regime the bench times.
steady_ns = None
traces = glob.glob(str(src / "trace" / "**" / "*kernel_trace.csv"), recursive=True)
if traces:
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in csv.DictReader(open(traces[0]))
         if KERNEL in r["Kernel_Name"]]
    if d:
        k0, acc = len(d) // 4, 0
        while k0 < len(d) - 1 and sum(d[:k0]) < 30e6:
            k0 += 1
        steady_ns = sum(d[k0:]) / len(d[k0:])
        lines.append(f"kernel_trace_steady_average_ns {steady_ns:.1f} (dispatches {k0 + 1}..{len(d)} of {len(d)}: "
                     "after the clock ramp)")
# Chained launches (bench.py's diffuse steps) overlap: each launch's own duration is longer
# than the step.  The comparable figure is the span of the longest run of overlapping or back-to-back
# dispatches of the instance (start of the next <= end of the previous + 20 us, i.e. no host
# synchronisation between them) divided by its number of dispatches.
span_ns = None
if traces:
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(traces[0]))
                if KERNEL in r["Kernel_Name"])
    runs, cur = [], [ev[0]] if ev else []
    for a, b in ev[1:]:
        if a <= max(e for _, e in cur[-2:]) + 20000:
            cur.append((a, b))
        else:
            runs.append(cur)
            cur = [(a, b)]
    if cur:
        runs.append(cur)
    # the longest run whose every dispatch started before its predecessor ended (the timed steps:
    # bench.py's K chained launches); none such (plain launches): the longest run
    ovl = [r for r in runs if all(r[i][0] < r[i - 1][1] for i in range(1, len(r)))]
    if runs:
        best = max(ovl or runs, key=len)
        n_ovl = sum(1 for i in range(1, len(best)) if best[i][0] < best[i - 1][1])
        span_ns = (max(b for _, b in best) - best[0][0]) / len(best)
        lines.append(f"kernel_trace_run_span_per_launch_ns {span_ns:.1f} (longest run of {len(best)} back-to-back "
                     f"dispatches, {n_ovl} of them starting before their predecessor ended)")
        if ovl:
            own = sum(b - a for a, b in best) / len(best)
            lines.append(f"kernel_trace_overlapped_own_duration_ns {own:.1f} (each launch's own start..end in that run)")
(dst / f"{tag}_pmc.txt").write_text("\n".join(lines) + "\n")
out = {"source": f"profiles/{tag}_pmc.txt", "workload": workload, "kernel": KERNEL, "kernel_average_ns": avg_ns,
       "kernel_steady_average_ns": steady_ns, "kernel_run_span_per_launch_ns": span_ns}
if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
    out["fetch_kib"] = mean["FETCH_SIZE"]
    out["write_kib"] = mean["WRITE_SIZE"]
    out["hbm_bytes_per_launch"] = (mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024.0
    out["hbm_bytes_per_launch_if_fetch_doubled"] = (2.0 * mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024.0
    out["note"] = ("bytes = (FETCH_SIZE + WRITE_SIZE) KiB; the x2 FETCH correction of the guide applies to "
                   "16-B/lane reads, not to this kernel's 12-B/lane accumulator reads (see script header)")
# VALU issue: wave-instructions per launch (SQ_INSTS_VALU is per wave, summed over the chip) over
# the kernel-trace duration and the 1024 SIMDs (256 CUs x 4) -> wave-instructions per SIMD per ns;
# the microbenchmarked ceiling is ~1.0 for 2-cycle ops, ~0.58 for the 4-cycle class
for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVES"):
    if k in mean:
        out[k.lower() + "_per_launch"] = mean[k]
if "SQ_INSTS_VALU" in mean and (steady_ns or avg_ns):
    out["valu_wave_insts_per_simd_per_ns"] = mean["SQ_INSTS_VALU"] / ((steady_ns or avg_ns) * 1024.0)
(dst / SUMMARY).write_text(json.dumps(out, indent=1) + "\n")
print("\n".join(lines))
print(json.dumps(out, indent=1))
