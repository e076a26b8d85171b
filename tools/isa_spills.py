#!/usr/bin/env python3
"""Where a kernel spills: parse a `hipcc --cuda-device-only -S -gline-tables-only`
listing, find one kernel, and count its scratch loads / stores by the source
line (.loc) they were emitted under, plus the kernel's VGPR / scratch totals.

    python tools/isa_spills.py f64g.s _ZN3rtw3dev13render_kernelIdLi5ELi0EEEvNS_7KParamsIT_EE
"""
import collections
import re
import sys


def main(path, sym, top=40):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    files = {}
    for l in lines:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
        if m:
            files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
    loc = "?"
    st, ld = collections.Counter(), collections.Counter()
    n_valu = 0
    for l in lines[start:end]:
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
        if m:
            loc = f"{files.get(m.group(1), m.group(1))}:{m.group(2)}"
            continue
        t = l.strip()
        if t.startswith("scratch_store") or t.startswith("buffer_store") and "off, s[0:3]" in t:
            st[loc] += 1
        elif t.startswith("scratch_load"):
            ld[loc] += 1
        elif t.startswith("v_"):
            n_valu += 1
    meta = {}
    for l in lines[end:end + 200]:
        m = re.match(r"\s*\.set\s+" + re.escape(sym) + r"\.(\w+),\s*(\S+)", l)
        if m:
            meta[m.group(1)] = m.group(2)
        m = re.match(r"\s*;\s*(NumVgprs|ScratchSize|Occupancy|NumVGPRsForWavesPerEU|VGPRBlocks):\s*(\S+)", l)
        if m:
            meta[m.group(1)] = m.group(2)
    print(f"{sym}: {sum(st.values())} scratch stores, {sum(ld.values())} scratch loads (static), "
          f"{n_valu} VALU; {meta}")
    both = collections.Counter()
    for k, v in st.items():
        both[k] += v
    for k, v in ld.items():
        both[k] += v
    for k, v in both.most_common(top):
        print(f"  {k:40s} stores {st[k]:4d} loads {ld[k]:4d}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *(int(a) for a in sys.argv[3:]))
