#!/usr/bin/env python3
"""CPU-baseline calibration against the reference's published probe figures.

SURVEY §6 timed the patched reference (flang -O2 -fopenmp, stand-in hull, 8 Xeon cores of this
container) on a GJK-only set: 32+32-vertex pairs that the sphere pre-test passes but GJK reports
separated, so neither EPA nor the hull stand-in runs: 0.067 M pairs/s on 1 core, ~0.45 M on 8.
This times the oracle restatement (oracle/gjkepa_oracle.c, the bench's cpu_baseline "port") on the
same kind of set in the same container and prints the ratios, so the GPU-vs-CPU figure of the bench
line can be read against the reference itself.  Set: the C2 generator with centre offset r up to 3,
keeping the pairs whose hull centres are 2..2.95 apart (inside the sphere test's +1.0 slack) and
that GJK reports separated.
usage: python tools/cpu_calib.py [n_pairs]  (prints one JSON line)"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "collision-detect-gjk-epa_amd"), os.path.join(ROOT, "oracle")]
import gjkepa  # noqa: E402
import oracle  # noqa: E402

REF_1CORE, REF_8CORE = 0.067, 0.45   # M pairs/s, SURVEY.md §6 (reference, GJK-only, this container)


def gjk_only_set(n: int):
    pool = gjkepa.synth_pairs(0x5EC0, 3 * n, 32, 32, 3.0)
    cen = np.stack([pool.verts[pool.hull_off[h]:pool.hull_off[h] + 96].reshape(3, 32).mean(axis=1)
                    for h in range(2 * pool.n_pairs)])
    d = np.linalg.norm(cen[1::2] - cen[0::2], axis=1)
    cand = gjkepa.HullPool(pool.verts, pool.hull_off, pool.hull_cnt, pool.pairs[np.nonzero((d > 2.0) & (d < 2.95))[0]])
    miss = oracle.gjkepa_batch(cand, 2, 1.0, 8)["collision"] == 0          # separated: GJK's miss
    return gjkepa.HullPool(pool.verts, pool.hull_off, pool.hull_cnt, cand.pairs[np.nonzero(miss)[0][:n]])


def rate(sub, threads: int, reps: int = 3) -> float:
    best = 0.0
    for _ in range(reps):
        t = time.perf_counter()
        oracle.gjkepa_batch(sub, 2, 1.0, threads)
        best = max(best, sub.n_pairs / (time.perf_counter() - t) / 1e6)
    return best


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
    sub = gjk_only_set(n)
    recs = oracle.gjkepa_batch(sub, 2, 1.0, 8)
    assert not recs["collision"].any(), "GJK-only set must be all misses"
    r1 = rate(gjkepa.HullPool(sub.verts, sub.hull_off, sub.hull_cnt, sub.pairs[:n // 8]), 1)
    r8 = rate(sub, 8)
    print(json.dumps({"set": f"{sub.n_pairs} separated 32+32-vertex pairs inside the sphere pre-test (GJK only)",
                      "port_1core": round(r1, 4), "port_8core": round(r8, 4),
                      "reference_1core": REF_1CORE, "reference_8core": REF_8CORE,
                      "port_over_reference_1core": round(r1 / REF_1CORE, 2),
                      "port_over_reference_8core": round(r8 / REF_8CORE, 2),
                      "cpu": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": \t"),
                      "nproc": os.cpu_count()}))


if __name__ == "__main__":
    main()
