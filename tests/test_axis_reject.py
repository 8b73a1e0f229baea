"""The GJK kernels' centre-axis quick reject: a pair whose hulls the axis between
their centres separates by more than the margin gets the reference's miss record without running
GJK.  These cases sit on both sides of that margin — touching, 1e-9 to 1e-5 gaps, overlaps of the
same size — at three length scales, with the gap along the centre axis and off it, and must equal
the oracle (the reference's GJK restated) byte for byte; the warm entry's misses likewise."""
import numpy as np
import pytest

import gjkepa

CUBE = np.array([[x, y, z] for z in (0, 1) for y in (0, 1) for x in (0, 1)], float)


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
