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


# --traffic OUT.json: HBM bytes per render_kernel launch from FETCH_SIZE /
# WRITE_SIZE (KB), corrected per MI355X_MICROARCH.md "HBM": FETCH_SIZE counts
# 64 B per 128-B request on gfx950 -> x2; WRITE_SIZE is exact.  bench.py
# reports it as roofline.traffic for the same kernel.
if len(sys.argv) > 3 and sys.argv[2] == "--traffic":
    import json
    fetch = sum(agg["FETCH_SIZE"]) / len(agg["FETCH_SIZE"]) * 1024 * 2
    write = sum(agg["WRITE_SIZE"]) / len(agg["WRITE_SIZE"]) * 1024
    names = set()
    for f in glob.glob(f"{root}/pmc*/pmc_counter_collection.csv"):
        for row in csv.DictReader(open(f)):
            if "render_kernel" in row["Kernel_Name"]:
                names.add(row["Kernel_Name"])
    json.dump({"kernel": sorted(names), "fetch_bytes": fetch, "write_bytes": write,
               "bytes_per_launch": fetch + write, "source": root,
               "correction": "FETCH_SIZE x2 (gfx950 64 B per 128-B request), WRITE_SIZE exact; KB units"},
              open(sys.argv[3], "w"), indent=1)
