#!/usr/bin/env python3
"""GPU box: the fp32-compute path on full batches against the fp64 path and against its CPU model.

Per config: GPU fp32 records vs GPU fp64 records (tools/fp32_metrics.py report), and vs the model of
the fp32 path on the CPU — the fp32 build of the oracle (oracle.gjkepa_batch_f32) whose uncertified
pairs (certificate flags in `reserved`, or an fp32 error status) are replaced by the fp64 records
rounded to fp32, which is what the GPU's redo launch computes.  Prints one JSON line per config.
usage: python tools/fp32_check.py [C2 C5 C4] [--pairs N]
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "collision-detect-gjk-epa_amd"), os.path.join(ROOT, "oracle"), ROOT,
                os.path.join(ROOT, "tools")]

import numpy as np  # noqa: E402

import gjkepa  # noqa: E402
import oracle  # noqa: E402
from bench import CONFIGS, SEED, host_cpus  # noqa: E402
from fp32_metrics import fp32_report  # noqa: E402


def model_fp32(pool, r64, threads):
    """CPU model of the GPU fp32 path: fp32 oracle, uncertified pairs from the fp64 records."""
    m = oracle.gjkepa_batch_f32(pool, 2, 1.0, threads)
    redo = (m["collision"] != 0) & ((m["reserved"] != 0) | (m["status"] == 1) | (m["status"] == 2))
    out = np.zeros(len(m), gjkepa.REC32)
    for f in ("penetration_depth", "collision_normal", "collision_point", "nearest_points", "collision",
              "colli_type", "status", "diag"):
        out[f] = np.where(redo.reshape((-1,) + (1,) * (m[f].ndim - 1)), r64[f], m[f])
    return out, redo


def main():
    cfgs = [a for a in sys.argv[1:] if a.startswith("C")] or ["C2", "C5", "C4"]
    npairs = int(sys.argv[sys.argv.index("--pairs") + 1]) if "--pairs" in sys.argv else 0
    threads = host_cpus()["usable"]
    for cfg in cfgs:
        nmin, nmax, rmax, n, _ = CONFIGS[cfg]
        n = npairs or n
        pool = gjkepa.synth_pairs(SEED, n, nmin, nmax, rmax, dtype=np.float32)
        g32 = gjkepa.gjkepa_batch(pool, 2, 1.0, gjkepa.PREC_F32)
        g64 = gjkepa.gjkepa_batch(pool, 2, 1.0, gjkepa.PREC_F64)
        rep = fp32_report(pool, g32, g64)
        model, redo = model_fp32(pool, g64, threads)
        eq = (g32.view(np.uint8).reshape(n, -1) == model.view(np.uint8).reshape(n, -1)).all(axis=1)
        rep.update({"config": cfg, "pairs": n, "model_redo_pairs": int(redo.sum()),
                    "bitexact_vs_cpu_model": float(eq.mean()), "mismatch_first": np.nonzero(~eq)[0][:8].tolist()})
        print(json.dumps(rep), flush=True)


if __name__ == "__main__":
    main()
