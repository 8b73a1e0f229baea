"""Separated-hull edge cases around the (diagnostic, off in the product) centre-axis quick reject
(DESIGN.md §4.1).  The reference's GJK can report a hit on hulls the axis between their centres
separates: the initial-simplex block (origin on the initial triangle's plane, :139-148) and the
tetrahedron loop's on-face branch (isPointInSimplex :1246-1256 + IS_INSIDE_PF :1271-1337, which
accepts a face lying in a coordinate plane through the origin).  The product therefore runs the
reference GJK on every pair.  These cases — touching, 1e-9 to 1e-5 gaps and overlaps at three length
scales, gaps along and off the centre axis, and boxes / prisms touching on one coordinate plane while
separated along another axis at rational offsets — must equal the oracle byte for byte, cold, with
fp32 storage, and through the warm entry (including a pair that missed last frame and whose next
frame is one of those on-face hits)."""
import numpy as np
import pytest

import gjkepa

CUBE = np.array([[x, y, z] for z in (0, 1) for y in (0, 1) for x in (0, 1)], float)
BOX = CUBE * [2, 1, 0.5]
PRISM = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [0, 0, 1], [1, 0, 1], [0, 1, 1]], float)


def ball(n, seed):
    rng = np.random.default_rng(seed)
    p = rng.normal(size=(n, 3))
    return p / np.linalg.norm(p, axis=1, keepdims=True)


def cases():
    out = []
    gaps = [-1e-5, -1e-6, -1e-9, 0.0, 1e-9, 1e-8, 5e-7, 1e-6, 1.5e-6, 3e-6, 1e-5, 1e-3]
    for s in (1e-3, 1.0, 1e3):
        for g in gaps:
            out.append((CUBE * s, (CUBE + [1 + g, 0.0, 0.0]) * s))           # face to face, on axis
            out.append((CUBE * s, (CUBE + [1 + g, 0.3, -0.2]) * s))          # offset: gap off the axis
            out.append((CUBE * s, (CUBE + [1 + g, 1 + g, 1 + g]) * s))       # corner to corner
        # one coordinate plane touching, another axis separated (the tetra loop's on-face hits)
        for o in [(-1, 0, 2), (-1, 1.25, 0), (1, 0, -2), (0, -1, 1.5), (1, 0.5, 1.25), (-1, -0.75, -2.5)]:
            out.append((CUBE * s, (CUBE + o) * s))
            out.append((BOX * s, (BOX + np.multiply(o, [2, 1, 0.5])) * s))
            out.append((PRISM * s, (PRISM + o) * s))
        a = ball(32, 7)
        for k, g in enumerate(gaps):
            u = ball(1, 100 + k)[0]
            b = ball(32, 200 + k)
            # centre distance chosen so the nearest projections along u are about g apart
            d = (a @ u).max() - (b @ u).min() + g
            out.append((a * s, (b + d * u) * s))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("version", [1, 2, 3])
def test_axis_reject_matches_oracle(orc, version):
    pool = gjkepa.HullPool.from_pairs(cases())
    g = gjkepa.gjkepa_batch(pool, version, 1.0)
    r = orc.gjkepa_batch(pool, version, 1.0)
    assert g.tobytes() == r.tobytes()
    assert 0 < int((r["collision"] != 0).sum()) < len(r)
    _, cov = orc.gjkepa_batch_cov(pool, version, 1.0)
    assert int(((cov >> np.uint64(orc.BR["LOOP_ONFACE"])) & np.uint64(1)).sum()) >= 10   # the adversarial hits


@pytest.mark.gpu
def test_axis_reject_fp32_storage_matches_oracle(orc):
    pool = gjkepa.HullPool.from_pairs([(a.astype(np.float32), b.astype(np.float32)) for a, b in cases()],
                                      dtype=np.float32)
    g = gjkepa.gjkepa_batch(pool, 2, 1.0)
    r = orc.gjkepa_batch(pool, 2, 1.0)
    assert g.tobytes() == r.tobytes()


@pytest.mark.gpu
def test_axis_reject_warm_second_call_misses_match_oracle(orc):
    """Warm entry, second call on the same frame: every miss (now answered by the miss mark +
    centre axis, or by GJK) equals the oracle's record; hits keep the oracle's hit flag."""
    from test_warm import fresh_warm, run
    pool = gjkepa.HullPool.from_pairs(cases())
    r = orc.gjkepa_batch(pool, 2, 1.0)
    w = fresh_warm(pool.n_pairs)
    run(pool, w)
    b = run(pool, w)
    np.testing.assert_array_equal(b["collision"], r["collision"])
    miss = r["collision"] == 0
    assert b[miss].tobytes() == r[miss].tobytes()


@pytest.mark.gpu
def test_warm_miss_then_onface_hit(orc):
    """Frame 0: the cubes far apart (a clean miss, slot marked); frame 1: cube + (-1, 0, 2), which the
    reference calls a hit through the on-face branch.  The warm entry must report that hit."""
    from test_warm import fresh_warm, run
    frames = [gjkepa.HullPool.from_pairs([(CUBE * s, (CUBE + o) * s) for s in (1e-3, 1.0) for o in offs])
              for offs in ([(-5, 0, 9)] * 3, [(-1, 0, 2), (-1, 1.25, 0), (1, 0, -2)])]
    w = fresh_warm(frames[0].n_pairs)
    a = run(frames[0], w)
    assert not a["collision"].any()
    b = run(frames[1], w)
    r = orc.gjkepa_batch(frames[1], 2, 1.0)
    assert r["collision"].all()
    assert b.tobytes() == r.tobytes()
