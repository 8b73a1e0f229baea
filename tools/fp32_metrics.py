"""Error metrics of the fp32-compute path against fp64 records of the same pairs.

Shared by tests/test_gpu_parity.py (the full-batch gate), bench.py (the fp32_compute side line) and
tools/fp32_check.py.  fp64 records are the truth (byte-identical to the oracle).  Per pair that
fp64 answers as an OK hit:
  - status: the fp32 record must be an OK hit too;
  - depth: |d32 - d64| <= DEPTH_TOL * |d64| (the north star's 1e-6 relative);
  - normal: angle(n32, n64) <= ANGLE (1e-5 rad), or n32 is a minimum-depth direction itself (a tie): the
    support of the Minkowski difference along n32, h_M(n32) = max_a a.n32 - min_b b.n32 in fp64 over the
    exact (fp32-stored) vertices, is within TIE_REL * |d64| of the depth.  Two faces whose distances
    agree to within that (C5: 1.728548533 vs 1.728548527, 2.6 rad apart) are both right answers; only
    fp64 arithmetic can order them.
The fp32 chain meets this by its certificate (csrc/gk_common.h Tol<float>::CERT_*): an fp32 answer is
kept only when its support gap plus the fp32 noise of its evaluation is within 5e-7 of the depth, every
other pair is recomputed in fp64.  fp32 coordinates of unit-scale hulls resolve ~1e-7, so shallow pairs
(depth below ~1 at C2's scale) all take the fp64 recomputation.
"""
from __future__ import annotations

import numpy as np

DEPTH_TOL = 1e-6
ANGLE = 1e-5
TIE_REL = 1e-6


def support_gap(pool, pair_idx, normals, depth64):
    """h_M(n) - d64 for the given pairs (fp64, unit-normalised n)."""
    out = np.empty(len(pair_idx))
    for k, (p, n) in enumerate(zip(pair_idx, normals)):
        a = pool.hull(int(pool.pairs[p, 0]))
        b = pool.hull(int(pool.pairs[p, 1]))
        u = np.asarray(n, np.float64)
        u = u / np.linalg.norm(u)
        out[k] = (a @ u).max() - (b @ u).min() - float(depth64[k])
    return out


def fp32_report(pool, g, r, angle: float | None = None) -> dict:
    """g: fp32-compute records, r: fp64 records of the same pool (structured arrays); `angle`: the
    normal bound (default ANGLE)."""
    angle = ANGLE if angle is None else angle
    ok64 = (r["collision"] != 0) & (r["status"] == 0)
    both = ok64 & (g["collision"] != 0) & (g["status"] == 0)
    d64 = r["penetration_depth"].astype(np.float64)
    d32 = g["penetration_depth"].astype(np.float64)
    ad = np.where(both, np.abs(d32 - d64), 0.0)
    rel = ad / np.maximum(np.abs(d64), 1e-9)
    a = g["collision_normal"].astype(np.float64)
    b = r["collision_normal"].astype(np.float64)
    cos = np.sum(a * b, axis=1) / np.maximum(np.linalg.norm(a, axis=1) * np.linalg.norm(b, axis=1), 1e-300)
    ang = np.where(both, np.arccos(np.clip(cos, -1.0, 1.0)), 0.0)
    unit = ad / np.maximum(1.0, np.abs(d64))
    depth_bad = both & (ad > DEPTH_TOL * np.abs(d64))
    # every pair whose normal is off by more than a tenth of the bound is checked for a tie, so the
    # reported non-tie maximum is one (a tie 0.9 x the bound apart would otherwise count as a non-tie)
    wide = np.nonzero(ang > 0.1 * angle)[0]
    gaps = support_gap(pool, wide, a[wide], d64[wide]) if wide.size else np.zeros(0)
    tie = gaps <= TIE_REL * np.abs(d64[wide])
    ang_nontie = ang.copy()
    ang_nontie[wide[tie]] = 0.0
    q = (lambda x, p: float(np.quantile(x[both], p)) if both.any() else 0.0)
    return {
        "hit_agreement": float((g["collision"] == r["collision"]).mean()),
        "status_mismatch": int((ok64 & ~both).sum()),
        "depth_relerr_p999": q(rel, 0.999), "depth_relerr_max": float(rel.max()),
        "depth_abserr_max": float(ad.max()),
        "depth_err_over_max1d_max": float(unit.max()),
        "depth_out_of_tol": int(depth_bad.sum()),
        "normal_angle_rad_p999": q(ang, 0.999), "normal_angle_rad_max": float(ang.max()),
        "normal_angle_rad_max_nontie": float(ang_nontie.max()),
        "normal_ties": int((tie & (ang[wide] > angle)).sum()),
        "normal_tie_gap_max": float(gaps[tie].max()) if tie.any() else 0.0,
        "normal_out_of_tol": int((~tie & (ang[wide] > angle)).sum()),
        "gate": {"depth": f"|d32-d64| <= {DEPTH_TOL} |d64|",
                 "normal": f"angle <= {angle} rad, or h_M(n32) - d64 <= {TIE_REL} |d64| (tie)"},
    }


def passes(rep: dict) -> bool:
    return (rep["hit_agreement"] == 1.0 and rep["status_mismatch"] == 0 and rep["depth_out_of_tol"] == 0
            and rep["normal_out_of_tol"] == 0)
