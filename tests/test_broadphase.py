"""Device broad phase: the pair list a caller's `DO a; DO b = a+1` loop over
GJKEPA reduces to — every pair passing the reference's own first test,
RoughCollisionDetection_SphericalEnvelope (GCLIB_GJKEPA.f90:76-77, :1165-1188).

CPU: the oracle (uniform-grid candidates + the exact predicate) against an O(N^2) brute force on
the same arithmetic, including invalid hulls; host-side API checks.  GPU (-m gpu): the HIP
pipeline (sphere kernel, radix sort, sweep, pair sort) through the C-ABI, identical to the oracle's
list (same pairs, same ascending order) on small scenes, mixed hull sizes, fp64 storage, a
truncated list, the device-pointer entry, and the full-size 2^20-hull scene; then broad phase ->
narrow phase on the device against the oracle."""
import os

import numpy as np
import pytest

import gjkepa

N_FULL = 1 << 20
BOX_FULL = (N_FULL * 113 / 6) ** (1 / 3)   # ~4 pairs per hull at r = 1 + 1 + 1.0 reach


def brute(pool):
    n = pool.hull_cnt.size
    m = np.full((n, 3), np.nan)
    r = np.full(n, np.nan)
    for h in range(n):
        c = int(pool.hull_cnt[h])
        if 1 <= c <= gjkepa.MAX_HULL_VERTS:
            p = pool.hull(h)
            s = np.zeros(3)
            for i in range(c):          # sequential sums, as the reference's SUM
                s = s + p[i]
            m[h] = s / c
            d = p - m[h]
            r[h] = np.sqrt((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]).max()
    d = m[:, None, :] - m[None, :, :]
    dist = np.sqrt((d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2])
    ok = dist <= (r[:, None] + r[None, :]) + 1.0
    return np.argwhere(np.triu(ok, 1)).astype(np.int32)


def scene_with_invalid():
    s = gjkepa.synth_scene(5, 600, 4, 64, 12.0, dtype=np.float64)
    cnt = s.hull_cnt.copy()
    cnt[3] = 0                                   # empty hull
    cnt[7] = 300                                 # too large
    v = s.verts.copy()
    v[s.hull_off[11]] = np.nan                   # non-finite vertex
    return gjkepa.HullPool(v, s.hull_off, cnt, s.pairs)


SCENES = {
    "dense": lambda: gjkepa.synth_scene(1, 2000, 32, 32, 15.0),
    "sparse": lambda: gjkepa.synth_scene(2, 3000, 8, 40, 60.0),
    "mixed": lambda: gjkepa.synth_scene(3, 1500, 8, 256, 20.0),
    "f64": lambda: gjkepa.synth_scene(4, 1000, 16, 16, 10.0, dtype=np.float64),
    "invalid": scene_with_invalid,
    "one": lambda: gjkepa.synth_scene(6, 1, 8, 8, 1.0),
}


# ---------------------------------------------------------------- CPU
@pytest.mark.parametrize("name", sorted(SCENES))
def test_oracle_matches_brute_force(orc, name):
    pool = SCENES[name]()
    pr, n = orc.broadphase(pool.verts, pool.hull_off, pool.hull_cnt)
    want = brute(pool)
    assert n == len(want)
    np.testing.assert_array_equal(pr.reshape(-1, 2), want.reshape(-1, 2))
    if name == "invalid":
        assert not np.isin(pr, [3, 7, 11]).any()


def test_oracle_truncates_but_counts(orc):
    pool = SCENES["dense"]()
    full, n = orc.broadphase(pool.verts, pool.hull_off, pool.hull_cnt)
    part, n2 = orc.broadphase(pool.verts, pool.hull_off, pool.hull_cnt, max_pairs=10)
    assert n2 == n and np.array_equal(part, full[:10])


def test_broadphase_api_validation_without_gpu(lib):
    assert lib.gjkepa_broadphase_workspace_bytes(-1, 0) < 0
    assert lib.gjkepa_broadphase(7, None, 0, None, None, 1, None, 0, None, 0) == -1
    n = np.zeros(1, np.int64)
    assert lib.gjkepa_broadphase(0, None, 0, None, None, 0, None, 0, n.ctypes.data, 0) == 0 and n[0] == 0
    assert lib.gjkepa_broadphase_device(0, None, None, None, 5, None, 0, None, None, 0, None) == -1


def test_synth_scene_deterministic_and_in_box():
    a = gjkepa.synth_scene(9, 200, 8, 64, 50.0)
    b = gjkepa.synth_scene(9, 50, 8, 64, 50.0, first_hull=150)
    for k in range(50):
        assert np.array_equal(a.hull(150 + k), b.hull(k))
    c = np.array([a.hull(h).mean(0) for h in range(200)])
    assert c.min() > -1.01 and c.max() < 51.01


# ---------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(SCENES))
def test_broadphase_matches_oracle(orc, name):
    pool = SCENES[name]()
    g, n = gjkepa.broadphase(pool)
    r, m = orc.broadphase(pool.verts, pool.hull_off, pool.hull_cnt)
    assert n == m
    np.testing.assert_array_equal(g.reshape(-1, 2), r.reshape(-1, 2))


@pytest.mark.gpu
def test_broadphase_truncated_list(orc):
    pool = SCENES["dense"]()
    r, m = orc.broadphase(pool.verts, pool.hull_off, pool.hull_cnt)
    g, n = gjkepa.broadphase(pool, max_pairs=m // 3)
    assert n == m and len(g) == m // 3
    assert np.all(np.diff(g[:, 0].astype(np.int64) * (1 << 32) + g[:, 1]) > 0)   # still ascending, distinct
    assert set(map(tuple, g)) <= set(map(tuple, r))


@pytest.mark.gpu
def test_broadphase_device_api_and_narrow_phase(orc):
    import torch
    pool = gjkepa.synth_scene(12, 20000, 16, 48, 80.0)
    dev = torch.device("cuda", 0)
    t = {k: torch.from_numpy(v).to(dev) for k, v in dict(v=pool.verts, o=pool.hull_off, c=pool.hull_cnt).items()}
    cap = 200000
    pairs = torch.full((cap, 2), -1, dtype=torch.int32, device=dev)
    npair = torch.zeros(1, dtype=torch.int64, device=dev)
    wsb = gjkepa.broadphase_workspace_bytes(pool.hull_cnt.size, cap)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        gjkepa.broadphase_device(gjkepa.DTYPE_F32, t["v"].data_ptr(), t["o"].data_ptr(), t["c"].data_ptr(),
                                 pool.hull_cnt.size, pairs.data_ptr(), cap, npair.data_ptr(), ws.data_ptr(), wsb,
                                 s.cuda_stream)
    s.synchronize()
    n = int(npair.item())
    r, m = orc.broadphase(pool.verts, pool.hull_off, pool.hull_cnt)
    assert n == m and n < cap
    got = pairs[:n].cpu().numpy()
    np.testing.assert_array_equal(got, r)
    # the narrow phase on the broad phase's list (device-resident end to end)
    cand = gjkepa.HullPool(pool.verts, pool.hull_off, pool.hull_cnt, got)
    recs = gjkepa.gjkepa_batch(cand, 2, 1.0)
    ref = orc.gjkepa_batch(cand, 2, 1.0)
    assert recs.tobytes() == ref.tobytes()
    assert 0.05 < recs["collision"].mean() < 0.95


@pytest.mark.gpu
def test_broadphase_full_size_matches_oracle(orc):
    pool = gjkepa.synth_scene(0x6A4B5C1D, N_FULL, 32, 32, BOX_FULL)
    g, n = gjkepa.broadphase(pool, max_pairs=8 * N_FULL)
    r, m = orc.broadphase(pool.verts, pool.hull_off, pool.hull_cnt)
    assert n == m and 3 * N_FULL < n < 6 * N_FULL
    assert np.array_equal(g, r)
