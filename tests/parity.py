"""Record comparison used by the GPU parity tests, smoke() and the tools (checker side only)."""
from __future__ import annotations

import numpy as np

REAL_FIELDS = ("penetration_depth", "collision_normal", "collision_point", "nearest_points")


def compare(gpu: np.ndarray, ref: np.ndarray, rtol: float = 1e-6, atol: float = 1e-9) -> dict:
    """Hit flag / status / type exact; reals within rtol relative (atol floor), NaN == NaN."""
    n = len(ref)
    res = {"n": n}
    hit_bad = gpu["collision"] != ref["collision"]
    st_bad = gpu["status"] != ref["status"]
    ty_bad = gpu["colli_type"] != ref["colli_type"]
    real_bad = np.zeros(n, bool)
    bitexact = np.ones(n, bool)
    maxrel = 0.0
    for f in REAL_FIELDS:
        a = gpu[f].astype(np.float64).reshape(n, -1)
        b = ref[f].astype(np.float64).reshape(n, -1)
        both_nan = np.isnan(a) & np.isnan(b)
        diff = np.abs(a - b)
        lim = rtol * np.abs(b) + atol
        bad = ~((diff <= lim) | both_nan)
        real_bad |= bad.any(axis=1)
        same = (a == b) | both_nan
        bitexact &= same.all(axis=1)
        with np.errstate(invalid="ignore", divide="ignore"):
            rel = np.where(both_nan, 0.0, diff / np.maximum(np.abs(b), atol))
        if rel.size:
            maxrel = max(maxrel, float(np.nanmax(rel)))
    res["hit_mismatch"] = int(hit_bad.sum())
    res["status_mismatch"] = int(st_bad.sum())
    res["type_mismatch"] = int(ty_bad.sum())
    res["real_mismatch"] = int(real_bad.sum())
    res["bitexact_frac"] = float(bitexact.mean()) if n else 1.0
    res["max_rel"] = maxrel
    res["bad_idx"] = np.nonzero(hit_bad | st_bad | ty_bad | real_bad)[0][:20].tolist()
    res["hits"] = int((ref["collision"] != 0).sum())
    res["ok"] = not (hit_bad.any() or st_bad.any() or ty_bad.any() or real_bad.any())
    return res


def fmt(r: np.void) -> str:
    return (f"hit={int(r['collision'])} type={int(r['colli_type'])} st={int(r['status'])} "
            f"diag={int(r['diag']):#x} d={float(r['penetration_depth']):.17g} n={np.asarray(r['collision_normal']).tolist()} "
            f"cp={np.asarray(r['collision_point']).tolist()} np={np.asarray(r['nearest_points']).tolist()}")
