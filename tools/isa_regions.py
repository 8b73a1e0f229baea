#!/usr/bin/env python3
"""Static instruction counts between GK_STAMP markers (build with -DGJKEPA_DIAG_MARKERS -save-temps).
usage: python tools/isa_regions.py <gfx950 .s file> <kernel-name substring>"""
import collections
import re
import sys

NAMES = {0: "gjk.load", 1: "gjk.sphere", 2: "gjk.init", 3: "gjk.update_simplex", 4: "gjk.checks+inside",
         5: "gjk.store", 6: "gjk.route", 10: "epa.load", 11: "epa.iter1", 12: "epa.dir", 13: "epa.support",
         14: "epa.visible", 15: "epa.horizon", 16: "epa.compact", 17: "epa.cone", 18: "epa.term",
         19: "epa.nearest", 20: "epa.contact", 21: "epa.type", 22: "epa.store", 23: "epa.route"}
src = open(sys.argv[1]).read()
key = sys.argv[2]
funcs = re.split(r"\n(?=_ZN2gk\w+:)", src)
for f in funcs:
    m = re.match(r"(_ZN2gk\w+):", f)
    if not m or key not in m.group(1):
        continue
    cur = -1
    cnt = collections.defaultdict(collections.Counter)
    for line in f.split("\n"):
        t = line.strip()
        mm = re.search(r"GKMARK (\d+)", t)
        if mm:
            cur = int(mm.group(1))
            continue
        if not t or t.startswith((".", ";", "_")) or t.endswith(":"):
            continue
        op = t.split()[0]
        k = ("dpp" if "dpp" in t else "f64" if "f64" in op else "valu") if op.startswith("v_") else \
            "nop" if op.startswith("s_nop") else "wait" if op.startswith("s_waitcnt") else \
            "salu" if op.startswith("s_") else "lds" if op.startswith("ds_") else "vmem"
        cnt[cur][k] += 1
    print(m.group(1))
    # instructions are attributed to the marker that PRECEDES them, i.e. the region after that stamp
    for rid in sorted(cnt):
        c = cnt[rid]
        tot = sum(c.values())
        print(f"  after {str(NAMES.get(rid, rid)):20s} {tot:6d}  " + " ".join(f"{k}={v}" for k, v in sorted(c.items())))
