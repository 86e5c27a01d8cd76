"""Summarise rocprofv3 counter CSVs for the render kernel (non-COUNT instantiation)."""
import collections, csv, glob, sys
out = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(f"{out}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "pt_render_kernel<0, false>" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:28s} n={len(v):3d} mean={sum(v)/len(v):.4g}")
