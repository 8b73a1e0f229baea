#!/usr/bin/env python3
"""Targeted search for the reference branches the round-2 fixture search did not reach
(LOOP_CAP :186, LOOP_CYCLE :219-234, EPA_STOP_SHRINK :1005-1010, V2_OVERLAP :1399-1418), with the
oracle's branch bits (oracle/gjkepa_oracle.h ORC_BR_*).  Candidate pools are built directly as
fixed-size SoA hulls (vectorised), so millions of pairs run in minutes on the container's cores.
Families: near-flat hulls (z noise 1e-12..1e-5), hulls at 1e3..1e8 scale, hulls at 1e-8..1e-5 scale,
near-coincident vertex clusters, many-vertex spheres grazing each other, duplicated extreme vertices.
usage: python tools/branch_search.py [millions of pairs per family] -> prints hits per branch and
saves the found pairs to /tmp/branch_hits.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "collision-detect-gjk-epa_amd"), os.path.join(ROOT, "oracle")]
import gjkepa  # noqa: E402
import oracle  # noqa: E402

TARGET = ("LOOP_CAP", "LOOP_CYCLE", "EPA_STOP_SHRINK", "V2_OVERLAP")


def pool_of(A, B):
    """A, B: (n, nv, 3) float64 arrays -> HullPool with hull 2k = A[k], 2k+1 = B[k]."""
    n, nv, _ = A.shape
    H = np.empty((2 * n, 3, nv))
    H[0::2] = A.transpose(0, 2, 1)
    H[1::2] = B.transpose(0, 2, 1)
    verts = H.reshape(-1)
    off = np.arange(2 * n, dtype=np.int64) * 3 * nv
    cnt = np.full(2 * n, nv, np.int32)
    prs = np.arange(2 * n, dtype=np.int32).reshape(n, 2)
    return gjkepa.HullPool(verts, off, cnt, prs)


def fam(rng, name, n):
    nv = int(rng.integers(4, 13))
    A = rng.normal(size=(n, nv, 3))
    B = rng.normal(size=(n, nv, 3))
    off = rng.normal(size=(n, 1, 3))
    if name == "flat":
        e = 10.0 ** rng.uniform(-12, -5, size=(n, 1, 1))
        A[..., 2] *= e[..., 0]
        B[..., 2] *= e[..., 0]
        off[..., 2] *= 10.0 ** rng.uniform(-12, -4, size=(n, 1))
    elif name == "big":
        s = 10.0 ** rng.uniform(3, 8, size=(n, 1, 1))
        A *= s; B *= s; off *= s
    elif name == "small":
        s = 10.0 ** rng.uniform(-8, -5, size=(n, 1, 1))
        A *= s; B *= s; off *= s
    elif name == "cluster":      # vertices in two tight clusters per hull
        s = 10.0 ** rng.uniform(-9, -6, size=(n, 1, 1))
        A = np.where(rng.random((n, nv, 1)) < 0.5, 1.0, -1.0) * np.array([1.0, 0, 0]) + A * s
        B = np.where(rng.random((n, nv, 1)) < 0.5, 1.0, -1.0) * np.array([0, 1.0, 0]) + B * s
    elif name == "graze":        # unit spheres of many points, centres ~2 apart
        A /= np.linalg.norm(A, axis=2, keepdims=True)
        B /= np.linalg.norm(B, axis=2, keepdims=True)
        off = off / np.linalg.norm(off, axis=2, keepdims=True) * (2.0 + 10.0 ** rng.uniform(-9, -3, size=(n, 1, 1)) *
                                                                   rng.choice([-1.0, 1.0], size=(n, 1, 1)))
    elif name == "dup":          # extreme vertex of A repeated three times, B's facing feature an edge
        A[..., 1:] *= 3.0
        A[..., 0] = -1.0 - np.abs(A[..., 0])
        A[:, :3, :] = np.array([1.0, 0.0, 0.0]) + rng.normal(size=(n, 1, 3)) * 0.0
        B[..., 1:] *= 3.0
        B[..., 0] = 3.0 + np.abs(B[..., 0])
        B[:, 0, :] = [0.9, -0.5, 0.0]
        B[:, 1, :] = [0.9, 0.5, 0.0]
        rot = rng.normal(size=(n, 3, 3)) * 10.0 ** rng.uniform(-4, -1, size=(n, 1, 1)) + np.eye(3)
        B = np.einsum("nij,nvj->nvi", rot, B)
        off = rng.normal(size=(n, 1, 3)) * 0.03
    elif name in ("grid", "gridrot"):   # points of a 3x3x3 surface grid: ties, face-interior support points
        g = np.array([[x, y, z] for x in (0, 0.5, 1) for y in (0, 0.5, 1) for z in (0, 0.5, 1)
                      if 0.0 in (x, y, z) or 1.0 in (x, y, z)], float)
        sa = rng.choice([0.5, 1.0, 2.0], size=(n, 1, 3))
        sb = rng.choice([0.5, 1.0, 2.0], size=(n, 1, 3))
        A = g[None] * sa
        B = g[None] * sb
        if name == "gridrot":
            ang = rng.choice([0.0, 1e-3, 0.1, np.pi / 4], size=n)
            c, s_ = np.cos(ang), np.sin(ang)
            R = np.zeros((n, 3, 3)); R[:, 0, 0] = c; R[:, 0, 1] = -s_; R[:, 1, 0] = s_; R[:, 1, 1] = c; R[:, 2, 2] = 1
            B = np.einsum("nij,nvj->nvi", R, B)
        off = np.round(rng.uniform(-2.5, 1.0, size=(n, 1, 3)) * 4) / 4
    return A, B + off


def main():
    per = float(sys.argv[1]) if len(sys.argv) > 1 else 0.5
    rng = np.random.default_rng(20261017)
    bits = {name: oracle.BRANCHES.index(name) for name in TARGET}
    found = {name: [] for name in TARGET}
    fams = sys.argv[2].split(",") if len(sys.argv) > 2 else ["dup", "grid", "gridrot", "flat", "big", "small", "cluster", "graze"]
    for name in fams:
        total = 0
        while total < per * 1e6:
            n = 100000
            A, B = fam(rng, name, n)
            pool = pool_of(A, B)
            masks = np.zeros(n, np.uint64)
            for v in (2,):
                masks |= oracle.gjkepa_batch_cov(pool, v, 1.0, 8)[1]
            for t, b in bits.items():
                hit = np.nonzero((masks >> np.uint64(b)) & np.uint64(1))[0]
                for k in hit[:8 - len(found[t])]:
                    found[t].append((A[k], B[k]))
            total += n
        print(name, int(total), {t: len(v) for t, v in found.items()}, flush=True)
    np.savez("/tmp/branch_hits.npz", **{f"{t}_{i}_{ab}": p for t, v in found.items() for i, pr in enumerate(v)
                                        for ab, p in zip("ab", pr)})


if __name__ == "__main__":
    main()
