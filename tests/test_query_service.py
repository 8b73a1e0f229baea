"""gjkepa_query's resident service (csrc/gjkepa_capi.cpp "resident query service"): a persistent grid
answers single-pair calls (the reference's `CALL GJKEPA`, GCLIB_GJKEPA.f90:39-52) from host-mapped
request slots.  Every record must be the oracle's bit for bit:
  - hulls of 4..256 vertices (the three hull register depths of the one-wave path) and deep
    penetrations whose polytope outgrows the small first polytope (the restart with the last EPA tier's);
  - across the grid's idle drain and relaunch;
  - with more concurrent callers than request slots (the rest take the combining path)."""
import concurrent.futures as cf
import threading
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


def _traffic(stop_evt, qs, counter):
    """One caller thread: single-pair calls in a loop until stop_evt is set."""
    i = 0
    while not stop_evt.is_set():
        gjkepa.gjkepa(*qs[i % len(qs)])
        i += 1
    counter.append(i)


@pytest.mark.gpu
def test_stop_then_device_synchronize_returns_promptly(orc):
    """gjkepa_query_service_stop drains the grid: a device-wide synchronisation right after it does
    not wait for the service's idle timeout, and the next call relaunches the grid (include/gjkepa.h)."""
    import torch
    qs = _big_pairs(8, 31, 4, 40)
    for q in qs:
        gjkepa.gjkepa(*q)                  # grid resident now
    t = time.perf_counter()
    gjkepa.query_service_stop(0)
    t_stop = time.perf_counter() - t
    assert not gjkepa.query_service_resident(0)   # the grid's completion event, not a wall clock
    t = time.perf_counter()
    torch.cuda.synchronize()
    t_sync = time.perf_counter() - t
    assert t_stop < 0.5, t_stop
    assert t_sync < 0.05, f"synchronize after stop took {t_sync * 1e3:.2f} ms"
    got = [gjkepa.gjkepa(*q) for q in qs]  # relaunched
    _check(orc, qs, got)
    gjkepa.query_service_stop(-1)          # all devices; nothing running is fine too
    gjkepa.query_service_stop(-1)


@pytest.mark.gpu
def test_synchronize_bounded_under_sustained_queries():
    """Under steady single-pair traffic the grid never idles; its 20 ms residency bound still lets a
    device-wide synchronisation return (it would otherwise wait until the traffic stops)."""
    import torch
    qs = _big_pairs(32, 41, 4, 40)
    stop_evt, counts = threading.Event(), []
    th = [threading.Thread(target=_traffic, args=(stop_evt, qs, counts)) for _ in range(4)]
    for x in th:
        x.start()
    try:
        time.sleep(0.1)
        waits = []
        for _ in range(5):
            t = time.perf_counter()
            torch.cuda.synchronize()
            waits.append(time.perf_counter() - t)
            time.sleep(0.05)
    finally:
        stop_evt.set()
        for x in th:
            x.join()
    assert max(waits) < 0.25, waits
    assert sum(counts) > 100


@pytest.mark.gpu
def test_batches_finish_beside_sustained_queries(orc):
    """gjkepa_batch calls on the same device while other threads keep the service busy: every batch
    finishes (the grid's residency bound) and its records are the oracle's."""
    qs = _big_pairs(32, 43, 4, 40)
    pool = gjkepa.synth_pairs(0x6A4B5C1D, 20000, 32, 32, 2.5)
    ref = orc.gjkepa_batch(gjkepa.HullPool(pool.verts, pool.hull_off, pool.hull_cnt, pool.pairs[:2000]), 2, 1.0)
    stop_evt, counts = threading.Event(), []
    th = [threading.Thread(target=_traffic, args=(stop_evt, qs, counts)) for _ in range(8)]
    for x in th:
        x.start()
    times = []
    try:
        time.sleep(0.05)
        for _ in range(4):
            t = time.perf_counter()
            g = gjkepa.gjkepa_batch(pool, 2, 1.0, gjkepa.PREC_F64)
            times.append(time.perf_counter() - t)
            assert g[:2000].tobytes() == ref.tobytes()
    finally:
        stop_evt.set()
        for x in th:
            x.join()
    assert max(times) < 1.0, times
    assert sum(counts) > 100


def _checked_traffic(stop_evt, qs, out):
    """One caller thread: single-pair calls in a loop until stop_evt is set, keeping (index, contact)."""
    i = 0
    while not stop_evt.is_set():
        out.append((i % len(qs), gjkepa.gjkepa(*qs[i % len(qs)])))
        i += 1


@pytest.mark.gpu
def test_service_off_while_calls_in_flight(orc):
    """gjkepa_query_service_set(0) while four threads keep calling: a call in flight is
    answered by the draining grid or finishes through the combining path — none relaunches the grid — so
    a device-wide synchronisation right after the callers stop does not wait for a resident grid; every
    answer is the oracle's.  Turning the service back on brings the grid back."""
    import torch
    qs = _big_pairs(24, 47, 4, 40)
    stop_evt = threading.Event()
    outs = [[] for _ in range(4)]
    th = [threading.Thread(target=_checked_traffic, args=(stop_evt, qs, o)) for o in outs]
    for x in th:
        x.start()
    try:
        time.sleep(0.1)
        assert gjkepa.query_service_set(False) is True
        time.sleep(0.1)                        # calls keep coming: combined now
    finally:
        stop_evt.set()
        for x in th:
            x.join()
    # no grid left on the GPU (checked on the grid's own completion event), so a device-wide
    # synchronisation does not wait for one; its time is bounded loosely (a resident grid would hold it
    # for GJKEPA_SVC_IDLE_US = 2 ms at least)
    resident = gjkepa.query_service_resident(0)
    t = time.perf_counter()
    torch.cuda.synchronize()
    t_sync = time.perf_counter() - t
    try:
        assert not resident, "a service grid is still resident after gjkepa_query_service_set(0)"
        assert t_sync < 0.05, f"synchronize with the service off took {t_sync * 1e3:.2f} ms"
        got = [c for o in outs for _, c in o]
        idx = [k for o in outs for k, _ in o]
        assert len(got) > 50
        ref = {k: orc.gjkepa(*qs[k]) for k in set(idx)}
        bad = [j for j, (k, c) in enumerate(zip(idx, got)) if not _same(c, ref[k])]
        assert not bad, f"{len(bad)} mismatches"
    finally:
        assert gjkepa.query_service_set(True) is False
    _check(orc, qs[:4], [gjkepa.gjkepa(*q) for q in qs[:4]])
