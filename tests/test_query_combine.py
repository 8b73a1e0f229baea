"""gjkepa_query under the reference's call pattern: many threads calling the single-pair entry at
once (`!$OMP PARALLEL DO ... CALL GJKEPA`, GCLIB_GJKEPA.f90:9, :16, :55-60).  Every test runs on both
paths of the entry: the resident query service (default) and, with the service switched off
(gjkepa_query_service_set(0)), the combiner, which batches the queued pairs of concurrent callers
into one GPU launch per (version_, TOL_FF_).  Every caller must get exactly its own record, bit for
bit the oracle's, with versions and tolerances (NaN included) mixed across threads and pairs of
different hull sizes in one batch."""
import concurrent.futures as cf

import numpy as np
import pytest

import gjkepa


def _pairs(n, seed):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        na, nb = rng.integers(4, 40, size=2)
        a = rng.normal(size=(na, 3))
        a /= np.linalg.norm(a, axis=1, keepdims=True)
        b = rng.normal(size=(nb, 3))
        b /= np.linalg.norm(b, axis=1, keepdims=True)
        d = rng.normal(size=3)
        b += d / np.linalg.norm(d) * rng.uniform(0, 2.5)
        out.append((int(1 + i % 3), (1.0, 1e-3)[i % 2], a, b))
    return out


@pytest.fixture(params=["service", "combiner"], autouse=True)
def query_path(request):
    """Run the module's tests through the resident service and through the combiner."""
    if "gpu" not in request.keywords:
        yield request.param
        return
    prev = gjkepa.query_service_set(request.param == "service")
    try:
        yield request.param
    finally:
        gjkepa.query_service_set(prev)


def _same(c, r):
    return (c.collision == bool(r["collision"]) and c.colli_type == int(r["colli_type"]) and
            c.status == int(r["status"]) and
            np.array_equal(np.asarray(c.collision_normal), r["collision_normal"]) and
            np.array_equal(np.asarray(c.collision_point), r["collision_point"]) and
            c.penetration_depth == float(r["penetration_depth"]) and
            np.array_equal(np.asarray(c.nearest_points), r["nearest_points"].reshape(2, 3)))


@pytest.mark.gpu
@pytest.mark.parametrize("threads", [1, 16])
def test_concurrent_queries_match_oracle(orc, threads):
    qs = _pairs(600, 7 + threads)
    with cf.ThreadPoolExecutor(threads) as ex:
        got = list(ex.map(lambda q: gjkepa.gjkepa(q[0], q[1], q[2], q[3]), qs))
    bad = [i for i, (q, c) in enumerate(zip(qs, got)) if not _same(c, orc.gjkepa(q[0], q[1], q[2], q[3]))]
    assert not bad, f"{len(bad)} mismatches, first {bad[:5]}"


@pytest.mark.gpu
def test_concurrent_query_error_reaches_its_caller():
    ok = _pairs(64, 3)
    bad = np.zeros((300, 3))                    # above GJKEPA_MAX_HULL_VERTS: answered BAD_INPUT, not an API error

    def one(i):
        if i % 8 == 0:
            return gjkepa.gjkepa(2, 1.0, bad, ok[i][3])
        return gjkepa.gjkepa(ok[i][0], ok[i][1], ok[i][2], ok[i][3])
    with cf.ThreadPoolExecutor(8) as ex:
        got = list(ex.map(one, range(64)))
    for i, c in enumerate(got):
        if i % 8 == 0:
            assert c.status == gjkepa.STATUS_BAD_INPUT and not c.collision


@pytest.mark.gpu
def test_concurrent_queries_nan_tolerance(orc):
    """A NaN TOL_FF_ never equals itself: the combiner still moves the first queued pair into its
    batch (compared bit for bit) instead of leaving it queued forever.  Mixed versions,
    finite and NaN tolerances from 12 threads; every caller gets the oracle's record."""
    qs = [(v, t, a, b) for (v, _, a, b), t in zip(_pairs(240, 11), [1.0, float("nan"), 1e-3, float("nan")] * 60)]
    with cf.ThreadPoolExecutor(12) as ex:
        got = list(ex.map(lambda q: gjkepa.gjkepa(q[0], q[1], q[2], q[3]), qs))
    bad = [i for i, (q, c) in enumerate(zip(qs, got)) if not _same(c, orc.gjkepa(q[0], q[1], q[2], q[3]))]
    assert not bad, f"{len(bad)} mismatches, first {bad[:5]}"
