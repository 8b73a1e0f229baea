"""Warm start for persistent pairs: gjkepa_batch_warm_device carries each
pair's last GJK simplex between calls and skips GJK when it still encloses the origin.

Bars, against the oracle run on the same frame: a call with no warm data is byte-identical to
gjkepa_batch_device (the reference path runs unchanged); on the next frame (hull B moved by a small
step) the hit flag is bit-exact with the oracle's, every pair that is not warm-started (misses
included) is byte-identical to the oracle's record, and warm-started hits agree with the oracle's
depth and normal within the north-star 1e-6 relative (absolute floor 1e-9 for near-zero depths:
EPA's own convergence test is 1e-8 absolute, GCLIB_GJKEPA.f90:972-1004)."""
import numpy as np
import pytest

import gjkepa

pytestmark = pytest.mark.gpu
RTOL, ATOL = 1e-6, 1e-9


def moved(pool, delta, seed=5):
    """Hull B of every pair translated by a random vector of length `delta` (new pool, same layout)."""
    rng = np.random.default_rng(seed)
    v = pool.verts.astype(np.float64).copy()
    for k in range(pool.n_pairs):
        h = int(pool.pairs[k, 1])
        o, n = int(pool.hull_off[h]), int(pool.hull_cnt[h])
        d = rng.normal(size=3)
        d *= delta / np.linalg.norm(d)
        for j in range(3):
            v[o + j * n:o + (j + 1) * n] += d[j]
    return gjkepa.HullPool(v.astype(pool.verts.dtype), pool.hull_off, pool.hull_cnt, pool.pairs)


def run(pool, warm=None):
    import torch
    dev = torch.device("cuda", 0)
    t = {k: torch.from_numpy(np.ascontiguousarray(x)).to(dev) for k, x in
         dict(v=pool.verts, o=pool.hull_off, c=pool.hull_cnt, p=pool.pairs.reshape(-1)).items()}
    out = torch.zeros(pool.n_pairs * 128, dtype=torch.uint8, device=dev)
    wsb = gjkepa.workspace_bytes(pool.n_pairs)
    ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
    dt = gjkepa.DTYPE_F32 if pool.verts.dtype == np.float32 else gjkepa.DTYPE_F64
    args = (2, 1.0, dt, gjkepa.PREC_F64, t["v"].data_ptr(), t["o"].data_ptr(), t["c"].data_ptr(), t["p"].data_ptr(),
            pool.n_pairs, out.data_ptr(), ws.data_ptr(), wsb)
    if warm is None:
        gjkepa.gjkepa_batch_device(*args)
    else:
        gjkepa.gjkepa_batch_warm_device(*args, warm.data_ptr())
    torch.cuda.synchronize()
    return np.frombuffer(out.cpu().numpy().tobytes(), gjkepa.REC64)


def fresh_warm(n):
    """A first call's warm slots: every code 0xFFFFFFFF (int32 -1 on the device)."""
    import torch
    return torch.full((4 * n,), -1, dtype=torch.int32, device="cuda")


@pytest.mark.parametrize("lo,hi", [(32, 32), (8, 256)])
def test_cold_warm_call_is_bitexact(lo, hi):
    pool = gjkepa.synth_pairs(0x5EED, 20000, lo, hi, 2.5)
    w = fresh_warm(pool.n_pairs)
    a = run(pool)
    b = run(pool, w)
    assert a.tobytes() == b.tobytes()
    codes = w.cpu().numpy().view(np.uint32).reshape(-1, 4)
    hit = a["collision"] != 0
    assert np.all(codes[~hit, 0] == 0xFFFFFFFE) and np.all(codes[~hit, 1:] == 0xFFFFFFFF)   # miss mark
    ok = a["status"] == 0
    assert np.all(codes[hit & ok] != 0xFFFFFFFF)


@pytest.mark.parametrize("lo,hi,delta", [(32, 32, 1e-3), (32, 32, 2e-2), (8, 256, 1e-3)])
def test_next_frame_matches_oracle(orc, lo, hi, delta):
    pool0 = gjkepa.synth_pairs(0x5EED, 20000, lo, hi, 2.5)
    pool1 = moved(pool0, delta)
    w = fresh_warm(pool0.n_pairs)
    run(pool0, w)
    warm = run(pool1, w)
    ref = orc.gjkepa_batch(pool1, 2, 1.0)          # the reference restated, on the moved frame
    np.testing.assert_array_equal(warm["collision"], ref["collision"])
    np.testing.assert_array_equal(warm["status"], ref["status"])
    started = (warm["diag"] & 0xFF) == 0            # GJK skipped: EPA ran from last frame's simplex
    started &= warm["collision"] != 0
    cold = ~started                                 # everything else ran the reference path
    assert warm[cold].tobytes() == ref[cold].tobytes()
    m = started & (ref["status"] == 0)
    assert m.sum() > 0.5 * ((ref["collision"] != 0) & (ref["status"] == 0)).sum()   # most hits skip GJK
    dr, dw = ref["penetration_depth"][m], warm["penetration_depth"][m]
    assert np.all(np.abs(dw - dr) <= ATOL + RTOL * np.abs(dr)), np.max(np.abs(dw - dr))
    nr, nw = ref["collision_normal"][m], warm["collision_normal"][m]
    assert np.all(np.linalg.norm(nw - nr, axis=1) <= RTOL), np.max(np.linalg.norm(nw - nr, axis=1))
    np.testing.assert_array_equal(warm["colli_type"][m], ref["colli_type"][m])
    agree = np.mean(np.all(warm[m].view(np.uint8).reshape(m.sum(), -1)[:, :104] ==
                           ref[m].view(np.uint8).reshape(m.sum(), -1)[:, :104], axis=1))
    print(f"delta {delta}: {m.sum()} hits warm-started, byte-identical to the oracle {agree:.4f}, "
          f"max |ddepth| {np.max(np.abs(dw - dr)):.3g}")
