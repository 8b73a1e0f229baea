"""gjkepa_collide: the whole all-pairs GJKEPA loop over a hull pool in one C-ABI call — device
broad phase (RoughCollisionDetection_SphericalEnvelope, GCLIB_GJKEPA.f90:76-77) -> batched
narrow phase -> hit compaction (collision_ flag, :47).  Parity: the oracle's broad phase, the
oracle's GJKEPA on each candidate, and the hits kept in candidate order, bit-exact records."""
import numpy as np
import pytest

import gjkepa


def scene_with_invalid():
    s = gjkepa.synth_scene(5, 600, 4, 64, 12.0, dtype=np.float64)
    cnt = s.hull_cnt.copy()
    cnt[3] = 0
    cnt[7] = 300
    v = s.verts.copy()
    v[s.hull_off[11]] = np.nan
    return gjkepa.HullPool(v, s.hull_off, cnt, s.pairs)


SCENES = {
    "dense": lambda: gjkepa.synth_scene(1, 2000, 32, 32, 15.0),
    "sparse": lambda: gjkepa.synth_scene(2, 3000, 8, 40, 60.0),
    "mixed": lambda: gjkepa.synth_scene(3, 1500, 8, 256, 20.0),
    "f64": lambda: gjkepa.synth_scene(4, 1000, 16, 16, 10.0, dtype=np.float64),
    "invalid": scene_with_invalid,
}


def expected(orc, pool, version=2):
    cand, n = orc.broadphase(pool.verts, pool.hull_off, pool.hull_cnt)
    cand = cand.reshape(-1, 2)
    sub = gjkepa.HullPool(pool.verts, pool.hull_off, pool.hull_cnt, np.ascontiguousarray(cand.reshape(-1)))
    recs = orc.gjkepa_batch(sub, version, 1.0)
    hit = recs["collision"] != 0
    return cand[hit], recs[hit], n


def test_collide_validation_without_gpu(lib):
    import ctypes
    n = ctypes.c_int64(-5)
    assert lib.gjkepa_collide(2, 1.0, 0, 1, None, 0, None, None, 0, None, None, 0, ctypes.byref(n), None, 0) == 0
    assert n.value == 0                                  # empty pool: no device needed
    assert lib.gjkepa_collide(2, 1.0, 7, 1, None, 0, None, None, 1, None, None, 0, ctypes.byref(n), None, 0) < 0
    assert lib.gjkepa_collide(2, 1.0, 0, 1, None, 0, None, None, 1, None, None, 4, ctypes.byref(n), None, 0) < 0


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(SCENES))
def test_collide_matches_oracle(orc, name):
    pool = SCENES[name]()
    want_p, want_r, want_n = expected(orc, pool)
    pairs, recs, ncand = gjkepa.collide(pool)
    assert ncand == want_n
    np.testing.assert_array_equal(pairs, want_p)
    assert recs.tobytes() == want_r.tobytes()


@pytest.mark.gpu
def test_collide_truncated_list_counts_all(orc):
    pool = SCENES["dense"]()
    want_p, want_r, _ = expected(orc, pool)
    assert len(want_p) > 20
    pairs, recs, _ = gjkepa.collide(pool, max_contacts=20)
    np.testing.assert_array_equal(pairs, want_p[:20])
    assert recs.tobytes() == want_r[:20].tobytes()


@pytest.mark.gpu
def test_collide_overflows_first_candidate_guess(orc):
    """More than 8 candidates per hull: the entry re-runs the broad phase at the counted size."""
    pool = gjkepa.synth_scene(7, 400, 8, 8, 4.0)
    want_p, want_r, want_n = expected(orc, pool)
    assert want_n > max(8 * 400, 1024)
    pairs, recs, ncand = gjkepa.collide(pool)
    assert ncand == want_n
    np.testing.assert_array_equal(pairs, want_p)
    assert recs.tobytes() == want_r.tobytes()
