#!/usr/bin/env python3
"""Summarise rocprofv3 PMC csvs for the render kernel: per-dispatch averages."""
import collections, csv, glob, sys
root = sys.argv[1]
agg = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/pmc*/pmc_counter_collection.csv")):
    per = collections.defaultdict(float)
    for row in csv.DictReader(open(f)):
        if "render_kernel" not in row["Kernel_Name"]:
            continue
        per[(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
    for (d, name), v in per.items():
        agg[name].append(v)
for k in sorted(agg):
    v = agg[k]
    print(f"{k:32s} {sum(v)/len(v):.4e}  (n={len(v)})")
