"""gjkepa_query's resident service (csrc/gjkepa_capi.cpp "resident query service"): a persistent grid
answers single-pair calls (the reference's `CALL GJKEPA`, GCLIB_GJKEPA.f90:39-52) from host-mapped
request slots.  Every record must be the oracle's bit for bit:
  - hulls of 4..256 vertices (the three hull register depths of the one-wave path) and deep
    penetrations whose polytope outgrows the small first polytope (the restart with the last EPA tier's);
  - across the grid's idle drain and relaunch;
  - with more concurrent callers than request slots (the rest take the combining path)."""
import concurrent.futures as cf
import time

import numpy as np
import pytest

import gjkepa
from test_query_combine import _same


def _big_pairs(n, seed, lo=4, hi=256):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        na, nb = rng.integers(lo, hi + 1, size=2)
        a = rng.normal(size=(na, 3))
        a /= np.linalg.norm(a, axis=1, keepdims=True)
        b = rng.normal(size=(nb, 3)) * rng.uniform(0.3, 1.5)
        d = rng.normal(size=3)
        b += d / np.linalg.norm(d) * rng.uniform(0, 1.2)          # mostly deep overlaps
        out.append((int(1 + i % 3), (1.0, 1e-3)[i % 2], a, b))
    return out


def _check(orc, qs, got):
    bad = [i for i, (q, c) in enumerate(zip(qs, got)) if not _same(c, orc.gjkepa(q[0], q[1], q[2], q[3]))]
    assert not bad, f"{len(bad)} mismatches, first {bad[:5]}"


@pytest.mark.gpu
def test_service_hull_depths_and_polytope_restart(orc):
    qs = _big_pairs(160, 21)
    got = [gjkepa.gjkepa(*q) for q in qs]
    _check(orc, qs, got)
    assert sum(c.collision for c in got) > 100


@pytest.mark.gpu
def test_service_idle_drain_and_relaunch(orc):
    qs = _big_pairs(12, 5, 4, 40)
    got = []
    for i, q in enumerate(qs):
        got.append(gjkepa.gjkepa(*q))
        if i % 3 == 2:
            time.sleep(0.02)          # well past the service's idle timeout: the grid drains
    _check(orc, qs, got)


@pytest.mark.gpu
def test_service_more_callers_than_slots(orc):
    qs = _big_pairs(400, 9, 4, 64)
    with cf.ThreadPoolExecutor(96) as ex:
        got = list(ex.map(lambda q: gjkepa.gjkepa(*q), qs))
    _check(orc, qs, got)


@pytest.mark.gpu
def test_service_bad_sizes(orc):
    a = np.zeros((0, 3))
    b = np.random.default_rng(1).normal(size=(8, 3))
    c = gjkepa.gjkepa(2, 1.0, a, b)
    assert c.status == gjkepa.STATUS_BAD_INPUT and not c.collision
    big = np.random.default_rng(2).normal(size=(300, 3))
    c = gjkepa.gjkepa(2, 1.0, big, b)
    assert c.status == gjkepa.STATUS_BAD_INPUT and not c.collision
