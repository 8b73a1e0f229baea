#!/usr/bin/env python3
"""Where the C2 chain's EPA tail goes: per-launch kernel durations (gjkepa_launch_timing) of the full C2
batch and of subsets made of its longest-EPA pairs (oracle iteration counts, the checker only), so the
time of the tiers that serve few pairs (EPA tier 1: polytopes that outgrow tier 0) can be split into
per-pair latency (a single pair alone) and contention (the same pairs inside the full chain).
usage: python tools/tail_probe.py [out.json]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "collision-detect-gjk-epa_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)
import gjkepa  # noqa: E402
import oracle  # noqa: E402  (checker: iteration counts only)
from bench import CONFIGS, SEED, host_cpus  # noqa: E402


def subset(pool, idx):
    return gjkepa.HullPool(verts=pool.verts, hull_off=pool.hull_off, hull_cnt=pool.hull_cnt,
                           pairs=np.ascontiguousarray(pool.pairs[idx]))


def chain(pool, reps=3):
    for _ in range(2):
        gjkepa.gjkepa_batch(pool, 2, 1.0, gjkepa.PREC_F64)
    gjkepa.launch_timing(True)
    for _ in range(reps):
        gjkepa.gjkepa_batch(pool, 2, 1.0, gjkepa.PREC_F64)
    gjkepa.launch_timing(False)
    lt = gjkepa.launch_timing_read()
    last = int(lt["chain"].max())
    rows = []
    for r in lt[lt["chain"] == last]:
        rows.append({"kernel": r["kernel"].decode(), "tier": int(r["tier"]), "part": int(r["part"]),
                     "stream": int(r["stream"]), "start_ms": round(float(r["start_ms"]), 4),
                     "ms": round(float(r["end_ms"] - r["start_ms"]), 4)})
    t0 = min(r["start_ms"] for r in rows)
    for r in rows:
        r["start_ms"] = round(r["start_ms"] - t0, 4)
    return rows


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    nmin, nmax, rmax, n, _ = CONFIGS["C2"]
    pool = gjkepa.synth_pairs(SEED, n, nmin, nmax, rmax, dtype=np.float32)
    rec = np.frombuffer(oracle.gjkepa_batch(pool, 2, 1.0, host_cpus()["usable"]).tobytes(),
                        dtype=gjkepa.record_dtype(gjkepa.PREC_F64))
    it = ((rec["diag"] >> 8) & 0xFF).astype(np.int64)
    it[rec["collision"] == 0] = -1
    order = np.argsort(-it, kind="stable")
    res = {"iters_max": int(it.max()), "iters_gt": {t: int((it > t).sum()) for t in (28, 30, 32, 36, 40)}}
    cases = [("top1", order[:1]), ("top16", order[:16]), ("gt36", np.flatnonzero(it > 36)),
             ("gt28", np.flatnonzero(it > 28)), ("full", np.arange(n))]
    for name, idx in cases:
        rows = chain(subset(pool, np.sort(idx)))
        res[name] = {"pairs": int(len(idx)), "launches": rows}
        print(f"== {name}: {len(idx)} pairs", flush=True)
        for r in rows:
            print(f"  {r['kernel']:8s} t{r['tier']} p{r['part']} s{r['stream']} at {r['start_ms']:8.4f} {r['ms']:8.4f} ms",
                  flush=True)
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
