#!/usr/bin/env python3
"""Summarise rocprofv3 PMC csvs for the render kernel: per-dispatch averages
over the steady-state renders.  Left out: the first render-kernel dispatch of
each pass (the first render of a scene / camera runs in tile index order and
counts the tile costs with atomics -- not the schedule the timed steps run)
and any launch under a quarter of the largest one of a counter (a 2-spp pilot
render, tuning lpt_inline=0)."""
import collections, csv, glob, sys
root = sys.argv[1]
agg = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/pmc*/pmc_counter_collection.csv")):
    per = collections.defaultdict(float)
    for row in csv.DictReader(open(f)):
        if "render_kernel" not in row["Kernel_Name"]:
            continue
        per[(int(row["Dispatch_Id"]), row["Counter_Name"])] += float(row["Counter_Value"])
    first = min((d for d, _ in per), default=None)
    top = collections.defaultdict(float)
    for (d, name), v in per.items():
        top[name] = max(top[name], v)
    for (d, name), v in per.items():
        if d != first and v >= 0.25 * top[name]:
            agg[name].append(v)
for k in sorted(agg):
    v = agg[k]
    print(f"{k:32s} {sum(v)/len(v):.4e}  (n={len(v)})")


# --traffic OUT.json [WORKLOAD]: HBM bytes per render_kernel launch from
# FETCH_SIZE / WRITE_SIZE (KB), corrected per MI355X_MICROARCH.md "HBM":
# FETCH_SIZE counts 64 B per 128-B request on gfx950 -> x2; WRITE_SIZE is
# exact.  With the SQ counters present also the VALU picture (SIMD-32: one
# wave64 VALU instruction = 2 cycles; GRBM_GUI_ACTIVE sums the 8 XCDs):
#   valu_issue_frac   = SQ_INSTS_VALU x 2 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
#   lanes_active_frac = SQ_THREAD_CYCLES_VALU / (64 x SQ_INSTS_VALU)
#   wave_wait_frac    = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (waiting for an instruction to issue)
#   mem_wait_frac     = SQ_WAIT_ANY / SQ_WAVE_CYCLES (waiting on any s_waitcnt: memory, LDS)
# bench.py reports them in `roofline` for the same kernel.
if len(sys.argv) > 3 and sys.argv[2] == "--traffic":
    import json
    avg = lambda k: sum(agg[k]) / len(agg[k])
    d = {"source": root}
    if agg.get("FETCH_SIZE") and agg.get("WRITE_SIZE"):
        d["fetch_bytes"] = avg("FETCH_SIZE") * 1024 * 2
        d["write_bytes"] = avg("WRITE_SIZE") * 1024
        d["bytes_per_launch"] = d["fetch_bytes"] + d["write_bytes"]
        d["correction"] = "FETCH_SIZE x2 (gfx950 64 B per 128-B request), WRITE_SIZE exact; KB units"
    if agg.get("SQ_INSTS_VALU") and agg.get("GRBM_GUI_ACTIVE"):
        d["valu_issue_frac"] = round(avg("SQ_INSTS_VALU") * 2 / (1024 * avg("GRBM_GUI_ACTIVE") / 8), 4)
    if agg.get("SQ_THREAD_CYCLES_VALU") and agg.get("SQ_INSTS_VALU"):
        d["lanes_active_frac"] = round(avg("SQ_THREAD_CYCLES_VALU") / (64 * avg("SQ_INSTS_VALU")), 4)
    if agg.get("SQ_WAIT_INST_ANY") and agg.get("SQ_WAVE_CYCLES"):
        d["wave_wait_frac"] = round(avg("SQ_WAIT_INST_ANY") / avg("SQ_WAVE_CYCLES"), 4)
    if agg.get("SQ_WAIT_ANY") and agg.get("SQ_WAVE_CYCLES"):
        d["mem_wait_frac"] = round(avg("SQ_WAIT_ANY") / avg("SQ_WAVE_CYCLES"), 4)
    # where the wave-cycles go (the attribution passes of tools/profile.sh):
    # cycles issuing each instruction type and waiting, as shares of
    # SQ_WAVE_CYCLES, and the mean cycles an instruction of each memory kind
    # is outstanding (SQ_INST_LEVEL_* / SQ_INSTS_*, Little's law)
    if agg.get("SQ_WAVE_CYCLES"):
        wc = avg("SQ_WAVE_CYCLES")
        att = {}
        for k in ("SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_LDS",
                  "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_MISC", "SQ_ACTIVE_INST_FLAT", "SQ_WAIT_ANY",
                  "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS"):
            if agg.get(k):
                att[k.replace("SQ_", "").lower() + "_frac"] = round(avg(k) / wc, 4)
        for lvl, n in (("SQ_INST_LEVEL_VMEM", "SQ_INSTS_VMEM"), ("SQ_INST_LEVEL_LDS", "SQ_INSTS_LDS"),
                       ("SQ_INST_LEVEL_SMEM", "SQ_INSTS_SMEM")):
            if agg.get(lvl) and agg.get(n):
                att[n.replace("SQ_INSTS_", "").lower() + "_cycles_outstanding"] = round(avg(lvl) / avg(n), 1)
        if agg.get("SQ_INSTS_BRANCH") and agg.get("SQ_INSTS_VALU"):
            att["branches_per_valu"] = round(avg("SQ_INSTS_BRANCH") / avg("SQ_INSTS_VALU"), 4)
        if att:
            d["attribution"] = att
    d["pmc_source"] = root
    names = set()
    for f in glob.glob(f"{root}/pmc*/pmc_counter_collection.csv"):
        for row in csv.DictReader(open(f)):
            if "render_kernel" in row["Kernel_Name"]:
                names.add(row["Kernel_Name"])
    d["kernel"] = sorted(names)
    if len(names) != 1:
        sys.exit(f"--traffic needs exactly one render-kernel variant in the passes, found {sorted(names)}: "
                 "profile one mode per run (bench.py --no-modes [--precision f64])")
    # the machine code these counters belong to: bench.py attaches them to a
    # line only when the kernel that ran has the same hash (run this on the
    # box, right after the passes, against the library they ran)
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from ray_tracing_weekend_amd import isa
    d["isa_sha"] = {n: isa.kernel_isa_sha(isa.demangled_to_symbol(n)) for n in d["kernel"]
                    if isa.demangled_to_symbol(n)}
    if len(sys.argv) > 4:
        d["workload"] = sys.argv[4]
    json.dump(d, open(sys.argv[3], "w"), indent=1)
