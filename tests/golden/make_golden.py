"""Regenerates the committed golden fixtures tests/golden/*.npz (run from the repo root).

Each fixture holds data only: seeded inputs from the deterministic workload generator
(gjkepa_synth_pairs, SURVEY.md §8d distributions), the oracle's expected contact records for
version_ = 1, 2, 3, and an independent ground truth for every hit — the penetration depth and
normal of scipy Qhull's hull of the full Minkowski difference.  The reference itself could not be
run here, so these pin the CPU restatement and the GPU path to each other and
to geometry, not to reference-produced numbers.

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "collision-detect-gjk-epa_amd"), os.path.join(ROOT, "oracle")]

import gjkepa  # noqa: E402
import oracle  # noqa: E402

SEED = 0x6A4B5C1D
# name: (n_pairs, n_min, n_max, r_max, tol_ff)
SETS = {
    "c2_32v": (1024, 32, 32, 2.5, 1.0),
    "c4_mixed": (192, 8, 256, 2.5, 1.0),
    "c5_deep": (256, 32, 128, 0.3, 1.0),
}
CUBE_OFFSETS = [(0.5, 0.2, 0.1), (1, 0, 0), (1 + 1e-9, 0, 0), (0, 0, 1e-3), (0.5, 0.5, 0.1), (0.3, 0.2, 0.1),
                (0.9, 0.8, 0.7), (0.9, 0.25, 0), (3, 0, 0), (0, 0, 0), (0.3, 0.3, 0.3), (1, 1, 1)]


def unit_cube() -> np.ndarray:
    return np.array([[x, y, z] for z in (0, 1) for y in (0, 1) for x in (0, 1)], float)


def qhull_truth(pool: gjkepa.HullPool):
    from scipy.spatial import ConvexHull
    inside = np.zeros(pool.n_pairs, bool)
    depth = np.zeros(pool.n_pairs)
    normal = np.zeros((pool.n_pairs, 3))
    for k in range(pool.n_pairs):
        a, b = pool.hull(int(pool.pairs[k, 0])), pool.hull(int(pool.pairs[k, 1]))
        m = (a[:, None, :] - b[None, :, :]).reshape(-1, 3)
        eq = ConvexHull(m).equations
        j = int(np.argmax(eq[:, 3]))
        inside[k] = bool(np.all(eq[:, 3] <= 1e-12))
        depth[k] = -eq[j, 3]
        normal[k] = eq[j, :3]
    return inside, depth, normal


def save(name: str, pool: gjkepa.HullPool, tol_ff: float, with_qhull: bool = True):
    recs = {f"rec_v{v}": oracle.gjkepa_batch(pool, v, tol_ff).view(np.uint8).reshape(pool.n_pairs, -1)
            for v in (1, 2, 3)}
    extra = {}
    if with_qhull:
        ins, dep, nrm = qhull_truth(pool)
        extra = {"qhull_inside": ins, "qhull_depth": dep, "qhull_normal": nrm}
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), verts=pool.verts, hull_off=pool.hull_off,
                        hull_cnt=pool.hull_cnt, pairs=pool.pairs, tol_ff=np.float64(tol_ff), **recs, **extra)
    print(name, pool.n_pairs, "pairs", os.path.getsize(os.path.join(HERE, f"{name}.npz")), "bytes")


def main():
    cube = unit_cube()
    pool = gjkepa.HullPool.from_pairs([(cube, cube + np.array(o)) for o in CUBE_OFFSETS], dtype=np.float64)
    save("c1_cubes", pool, 1e-3, with_qhull=False)
    for name, (n, lo, hi, rmax, tol) in SETS.items():
        save(name, gjkepa.synth_pairs(SEED, n, lo, hi, rmax, dtype=np.float32), tol)


if __name__ == "__main__":
    main()
