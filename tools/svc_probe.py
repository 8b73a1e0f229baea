#!/usr/bin/env python3
"""Single-caller latency of gjkepa_query's resident service on C2-shaped pairs (32 + 32 vertices on
the unit sphere, hull B offset by r ~ U[0, 2.5]: the call-pattern benchmark's distribution).  Prints
us per call by outcome (miss / hit); with a -DGJKEPA_DIAG_STAMPS library (GJKEPA_LIB) also the
per-phase share of the serving wave's time.  usage: [GJKEPA_QUERY_STATS=1] python tools/svc_probe.py [n]"""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "collision-detect-gjk-epa_amd"))
import gjkepa  # noqa: E402

NAMES = {0: "gjk.load", 1: "gjk.sphere", 2: "gjk.init", 3: "gjk.update_simplex", 4: "gjk.checks+inside",
         10: "epa.load", 11: "epa.iter1", 12: "epa.dir", 13: "epa.support", 14: "epa.visible", 15: "epa.horizon",
         16: "epa.compact", 17: "epa.cone", 18: "epa.term", 19: "epa.nearest", 20: "epa.contact", 21: "epa.type"}


def pairs(n, seed=5):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        a = rng.normal(size=(32, 3))
        a /= np.linalg.norm(a, axis=1, keepdims=True)
        b = rng.normal(size=(32, 3))
        b /= np.linalg.norm(b, axis=1, keepdims=True)
        u = rng.normal(size=3)
        b += u / np.linalg.norm(u) * rng.uniform(0, 2.5)
        out.append((a, b))
    return out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    lib = gjkepa.load()
    stamps = hasattr(lib, "gjkepa_diag_stamps")
    qs = pairs(n)
    for a, b in qs[:50]:
        gjkepa.gjkepa(2, 1.0, a, b)
    if stamps:
        lib.gjkepa_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
        buf = np.zeros(32, dtype=np.uint64)
        lib.gjkepa_diag_stamps(buf.ctypes.data, 1)
    t = np.zeros(n)
    hit = np.zeros(n, bool)
    for i, (a, b) in enumerate(qs):
        t0 = time.perf_counter()
        c = gjkepa.gjkepa(2, 1.0, a, b)
        t[i] = time.perf_counter() - t0
        hit[i] = c.collision
    us = 1e6 * t
    print(f"{n} calls: {us.mean():.1f} us/call (python included); miss {us[~hit].mean():.1f} ({(~hit).sum()}), "
          f"hit {us[hit].mean():.1f} ({hit.sum()}); p50 {np.median(us):.1f} p90 {np.percentile(us, 90):.1f}")
    if stamps:
        lib.gjkepa_diag_stamps(buf.ctypes.data, 1)
        tot = float(buf.sum())
        print(f"serving wave: {tot / n:.0f} ticks per call")
        for i in range(32):
            if buf[i]:
                print(f"  {NAMES.get(i, str(i)):22s} {100 * buf[i] / tot:5.1f}%  {buf[i] / n:8.0f} ticks/call")


if __name__ == "__main__":
    main()
