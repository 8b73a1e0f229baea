"""Full-size (BASELINE C2: 2^20 pairs) GPU checks through size-independent properties, plus a
random subsample compared byte for byte with the oracle."""
import numpy as np
import pytest

import gjkepa

pytestmark = pytest.mark.gpu
N = 1 << 20


@pytest.fixture(scope="module")
def c2_full():
    pool = gjkepa.synth_pairs(0x6A4B5C1D, N, 32, 32, 2.5)
    return pool, gjkepa.gjkepa_batch(pool, 2, 1.0)


def test_deterministic_across_runs(c2_full):
    pool, a = c2_full
    b = gjkepa.gjkepa_batch(pool, 2, 1.0)
    assert a.tobytes() == b.tobytes()


def test_subsample_bitexact_vs_oracle(c2_full, orc):
    pool, g = c2_full
    idx = np.sort(np.random.default_rng(1).choice(N, 8192, replace=False))
    sub = gjkepa.HullPool(pool.verts, pool.hull_off, pool.hull_cnt, pool.pairs[idx])
    r = orc.gjkepa_batch(sub, 2, 1.0)
    assert g[idx].tobytes() == r.tobytes()


def test_record_invariants(c2_full):
    _, g = c2_full
    hit = g["collision"] != 0
    ok = g["status"] == 0
    assert ok.mean() > 0.999
    assert 0.6 < hit.mean() < 0.85                                      # ~73% hits at r ~ U[0, 2.5]
    miss = ~hit
    assert not np.any(g["penetration_depth"][miss]) and not np.any(g["collision_normal"][miss])
    assert np.all(g["colli_type"][miss] == 0)
    h = hit & ok
    assert np.all(g["penetration_depth"][h] >= 0)
    assert np.allclose(np.linalg.norm(g["collision_normal"][h], axis=1), 1, atol=1e-12)
    assert set(np.unique(g["colli_type"][h]).tolist()) <= {1, 2}
    # depth is the support-gap along n: max_i n.a_i - min_j n.b_j for the nearest points
    npts = g["nearest_points"][h]
    gap = np.einsum("ij,ij->i", g["collision_normal"][h], npts[:, :3] - npts[:, 3:])
    assert np.allclose(gap, g["penetration_depth"][h], atol=1e-9)


def test_fp32_storage_equals_fp64_storage(c2_full):
    pool, g = c2_full
    sub = gjkepa.HullPool(pool.verts.astype(np.float64), pool.hull_off, pool.hull_cnt, pool.pairs[:100000])
    assert gjkepa.gjkepa_batch(sub, 2, 1.0).tobytes() == g[:100000].tobytes()
