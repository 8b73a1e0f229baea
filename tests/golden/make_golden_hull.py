"""Regenerates tests/golden/h1_clouds.npz, the fixture of the batched hull module (SURVEY.md §8
row f1), from the repo root:

    python tests/golden/make_golden_hull.py

Data only: seeded point clouds (gjkepa_synth_clouds ball / sphere clouds of 4..256 points plus
hand-made edge cases: cube corners with face-centre and interior points, duplicated points, a
4x4x4 grid, scaled clouds, flat / collinear / coincident / too small / too large / non-finite
clouds), the oracle's outputs (oracle_hull_batch: faces, counts, vertex indices, statuses), and an
independent ground truth from scipy Qhull (hull vertex set and volume) for every cloud it accepts.
The reference's GCLIB_QuickHull is unvendored, so this pins the restatement and the
GPU path to each other and to geometry, not to reference-produced numbers.
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


def edge_clouds():
    rng = np.random.default_rng(SEED)
    cube = np.array([[x, y, z] for z in (0, 1) for y in (0, 1) for x in (0, 1)], float)
    centres = np.array([[.5, .5, 0], [.5, .5, 1], [.5, 0, .5], [.5, 1, .5], [0, .5, .5], [1, .5, .5]])
    grid = np.stack(np.meshgrid(*[np.arange(4.0)] * 3, indexing="ij"), -1).reshape(-1, 3)
    ball = rng.normal(size=(40, 3))
    out = [
        np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [0, 0, 1.0]]),             # tetrahedron
        cube,                                                                   # coplanar faces
        np.concatenate([cube, centres, rng.uniform(0.2, 0.8, (20, 3))]),       # + coplanar + interior
        np.concatenate([ball, ball]),                                           # every point twice
        grid,                                                                   # 4x4x4 lattice
        1e3 * rng.normal(size=(50, 3)),                                         # large scale
        1e-3 * rng.normal(size=(50, 3)),                                        # small scale
        np.c_[rng.normal(size=(30, 2)), np.zeros(30)],                          # flat -> DEGENERATE
        np.outer(rng.normal(size=20), [1.0, 2.0, 3.0]),                         # collinear -> DEGENERATE
        np.ones((10, 3)),                                                       # coincident -> DEGENERATE
        rng.normal(size=(3, 3)),                                                # n < 4 -> BAD_INPUT
        rng.normal(size=(257, 3)),                                              # n > 256 -> BAD_INPUT
        np.r_[rng.normal(size=(9, 3)), [[np.nan, 0, 0]]],                       # non-finite -> BAD_INPUT
    ]
    return [np.asarray(p, np.float32).astype(np.float64) for p in out]


def clouds():
    lst = edge_clouds()
    for shape in (0, 1):
        for lo, hi, n in ((4, 16, 48), (17, 64, 48), (65, 256, 24)):
            pool = gjkepa.synth_clouds(SEED + shape, n, lo, hi, shape, dtype=np.float32)
            lst += [pool.cloud(c) for c in range(pool.n_clouds)]
    return lst


def qhull_truth(pool: gjkepa.CloudPool, status):
    """Per OK cloud: sorted hull vertex indices and volume from scipy Qhull (-1 / NaN otherwise)."""
    from scipy.spatial import ConvexHull
    vidx = np.full(pool.verts.size, -1, np.int32)
    vol = np.full(pool.n_clouds, np.nan)
    for c in range(pool.n_clouds):
        if status[c] != 0:
            continue
        h = ConvexHull(pool.cloud(c))
        v = np.sort(h.vertices)
        vidx[pool.cloud_off[c]:pool.cloud_off[c] + len(v)] = v
        vol[c] = h.volume
    return vidx, vol


def main():
    pool = gjkepa.CloudPool.from_list(clouds(), dtype=np.float64)
    r = oracle.hull_batch(pool.verts, pool.cloud_off, pool.cloud_cnt)
    qv, qvol = qhull_truth(pool, r["status"])
    path = os.path.join(HERE, "h1_clouds.npz")
    np.savez_compressed(path, verts=pool.verts, cloud_off=pool.cloud_off, cloud_cnt=pool.cloud_cnt,
                        faces=r["faces"], face_off=r["face_off"], n_faces=r["n_faces"], n_verts=r["n_verts"],
                        status=r["status"], vert_idx=r["vert_idx"], qhull_vert_idx=qv, qhull_volume=qvol)
    print("h1_clouds", pool.n_clouds, "clouds; statuses", np.bincount(r["status"]), os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
