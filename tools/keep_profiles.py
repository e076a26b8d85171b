#!/usr/bin/env python3
"""Copy one GPU session's results from gpurun_out/ into profiles/ under the
round's names (what the judge reads):
  tools/keep_profiles.py TAG      (TAG as given to tools/gpu_round.sh, e.g. r03_v0)
pytest log, bench line, kernel-trace stats and, per profiled kernel, the PMC
summary + traffic JSON (its `source` rewritten to the committed summary)."""
import glob
import json
import os
import shutil
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
G, P = os.path.join(ROOT, "gpurun_out"), os.path.join(ROOT, "profiles")
tag = sys.argv[1]


def cp(src, dst):
    if os.path.exists(src):
        shutil.copyfile(src, os.path.join(P, dst))
        print("kept", dst)


cp(f"{G}/pytest_gpu_{tag}.log", f"{tag}_pytest_gpu.log")
cp(f"{G}/bench_{tag}.json", f"{tag}_bench.json")
for sub in ("", "_f32", "_f64"):
    t = f"{tag}{sub}"
    stats = glob.glob(f"{G}/prof_{t}/*kernel_stats.csv")
    if stats:
        cp(stats[0], f"{t}_kernel_stats.csv")
    cp(f"{G}/prof_{t}_pmc_summary.txt", f"{t}_pmc_summary.txt")
    tj = f"{G}/prof_{t}_traffic.json"
    if os.path.exists(tj):
        d = json.load(open(tj))
        d["source"] = d["pmc_source"] = f"profiles/{t}_pmc_summary.txt"
        json.dump(d, open(os.path.join(P, f"{t}_traffic.json"), "w"), indent=1)
        print("kept", f"{t}_traffic.json")
