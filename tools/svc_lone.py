#!/usr/bin/env python3
"""GPU box: single-pair call latency through gjkepa_query (the reference's `CALL GJKEPA`, :39-52) from one
thread and from 16, on C2-distribution 32-vertex pairs, with every record checked against the oracle on
a subset.  GJKEPA_LIB selects the library (A/B of variants).  Prints one JSON line.
usage: python tools/svc_lone.py [n_calls]"""
from __future__ import annotations

import concurrent.futures as cf
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "collision-detect-gjk-epa_amd"), os.path.join(ROOT, "oracle"), ROOT]

import numpy as np  # noqa: E402

import gjkepa  # noqa: E402
from bench import SEED  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    pool = gjkepa.synth_pairs(SEED, n, 32, 32, 2.5)
    qs = [(2, 1.0, pool.hull(int(a)), pool.hull(int(b))) for a, b in pool.pairs]
    for q in qs[:50]:
        gjkepa.gjkepa(*q)                                   # service up
    t = time.perf_counter()
    one = [gjkepa.gjkepa(*q) for q in qs]
    lone_us = 1e6 * (time.perf_counter() - t) / n
    with cf.ThreadPoolExecutor(16) as ex:
        list(ex.map(lambda q: gjkepa.gjkepa(*q), qs[:200]))
        t = time.perf_counter()
        many = list(ex.map(lambda q: gjkepa.gjkepa(*q), qs))
        t16_us = 1e6 * (time.perf_counter() - t) / n
    import oracle  # checker only
    sub = np.arange(0, n, 7)
    ref = oracle.gjkepa_batch(gjkepa.HullPool(pool.verts, pool.hull_off, pool.hull_cnt, pool.pairs[sub]), 2, 1.0)
    bad = 0
    for k, i in enumerate(sub):
        for c in (one[i], many[i]):
            r = ref[k]
            bad += not (bool(c.collision) == bool(r["collision"]) and c.status == r["status"]
                        and c.penetration_depth == r["penetration_depth"]
                        and np.array_equal(c.collision_normal, r["collision_normal"]))
    print(json.dumps({"lib": gjkepa.version_string().rsplit("src ", 1)[-1], "calls": n, "lone_us_per_call": round(lone_us, 2),
                      "threads16_us_per_pair": round(t16_us, 3), "checked": int(2 * len(sub)), "mismatches": bad}))


if __name__ == "__main__":
    main()
