"""Batched convex hulls (GCLIB_QuickHull::QuickHull +
GCLIB_DeHull::getHullMeshesVertex, used at GCLIB_GJKEPA.f90:920, :950).

CPU: the oracle restatement against scipy Qhull ground truth (vertex set, volume, outward
supporting faces, Euler count) and against the committed fixture; host-side API checks.
GPU (-m gpu): the HIP kernels through the C-ABI, bit-exact against the oracle — faces and their
order, vertex indices, hull pools, statuses — on the fixture, on random clouds of every size
4..256 (both kernel tiers) and through the device-pointer entry; and the raw-cloud -> hull ->
narrow-phase workflow.  The reference's hull modules are unvendored, so parity with them is
unpinned; the pin is geometry (Qhull) plus oracle/GPU identity.
"""
import os

import numpy as np
import pytest

import gjkepa

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
OK, DEGENERATE, BAD_INPUT = gjkepa.STATUS_OK, gjkepa.STATUS_DEGENERATE, gjkepa.STATUS_BAD_INPUT


def fixture():
    z = np.load(os.path.join(GOLDEN, "h1_clouds.npz"))
    return z, gjkepa.CloudPool(z["verts"], z["cloud_off"], z["cloud_cnt"])


def check_geometry(p, faces, vidx, volume=None, vset=None):
    """Outward, supporting faces; closed (every directed edge has its twin); F = 2V - 4."""
    cen = p[vidx].mean(0)
    scale = np.abs(p).max()
    vol = 0.0
    edges = set()
    for a, b, c in faces:
        n = np.cross(p[b] - p[a], p[c] - p[b])
        assert np.dot(n, p[a] - cen) > 0
        assert ((p - p[a]) @ n).max() <= 1e-9 * np.linalg.norm(n) * max(scale, 1.0)
        vol += np.dot(p[a] - cen, np.cross(p[b] - cen, p[c] - cen)) / 6.0
        edges |= {(a, b), (b, c), (c, a)}
    assert all((w, u) in edges for (u, w) in edges)
    assert len(faces) == 2 * len(vidx) - 4
    assert set(np.unique(faces)) == set(vidx)
    if volume is not None:
        assert vol == pytest.approx(volume, rel=1e-9)
    if vset is not None:   # compare coordinates: duplicated points may be represented by either copy
        assert {tuple(x) for x in p[vidx]} == {tuple(x) for x in p[np.asarray(vset)]}


def per_cloud(r, pool, c):
    nf, nv, o = int(r["n_faces"][c]), int(r["n_verts"][c]), int(pool.cloud_off[c])
    return r["faces"][r["face_off"][c]:r["face_off"][c] + nf], r["vert_idx"][o:o + nv]


# ---------------------------------------------------------------- CPU: oracle and host side
def test_oracle_matches_fixture(orc):
    z, pool = fixture()
    r = orc.hull_batch(pool.verts, pool.cloud_off, pool.cloud_cnt)
    for k in ("faces", "face_off", "n_faces", "n_verts", "status"):
        np.testing.assert_array_equal(r[k], z[k], err_msg=k)
    np.testing.assert_array_equal(r["vert_idx"][z["vert_idx"] >= 0], z["vert_idx"][z["vert_idx"] >= 0])


def test_oracle_vs_qhull_ground_truth(orc):
    z, pool = fixture()
    r = orc.hull_batch(pool.verts, pool.cloud_off, pool.cloud_cnt)
    assert (r["status"] == OK).sum() >= 240
    for c in range(pool.n_clouds):
        if r["status"][c] != OK:
            continue
        faces, vidx = per_cloud(r, pool, c)
        o = int(pool.cloud_off[c])
        qv = z["qhull_vert_idx"][o:o + int(pool.cloud_cnt[c])]
        check_geometry(pool.cloud(c), faces, vidx, z["qhull_volume"][c], qv[qv >= 0])
        assert np.all(np.diff(vidx) > 0)                       # ascending point index


def test_oracle_edge_case_statuses(orc):
    z, pool = fixture()
    st = z["status"][:13]
    assert list(st[:7]) == [OK] * 7
    assert list(st[7:10]) == [DEGENERATE] * 3                  # flat, collinear, coincident
    assert list(st[10:13]) == [BAD_INPUT] * 3                  # n < 4, n > 256, NaN
    assert z["n_verts"][0] == 4 and z["n_faces"][0] == 4
    assert z["n_verts"][1] == 8 and z["n_faces"][1] == 12      # cube: corners only
    assert z["n_verts"][2] == 8                                # face centres / interior dropped
    assert z["n_verts"][4] == 8                                # lattice: its 8 corners
    assert np.all(z["n_faces"][7:13] == 0) and np.all(z["n_verts"][7:13] == 0)


def test_oracle_fresh_random_vs_qhull(orc):
    from scipy.spatial import ConvexHull
    pool = gjkepa.synth_clouds(99, 200, 4, 256, 0, dtype=np.float64)
    r = orc.hull_batch(pool.verts, pool.cloud_off, pool.cloud_cnt)
    assert np.all(r["status"] == OK)
    for c in range(0, pool.n_clouds, 3):
        p = pool.cloud(c)
        h = ConvexHull(p)
        faces, vidx = per_cloud(r, pool, c)
        check_geometry(p, faces, vidx, h.volume, h.vertices)


def test_hull_api_validation_without_gpu(lib):
    assert lib.gjkepa_hull_face_capacity(4) == 4 and lib.gjkepa_hull_face_capacity(256) == 508
    assert lib.gjkepa_hull_face_capacity(3) == 0
    assert lib.gjkepa_hull_batch(7, None, 0, None, None, 1, None, 0, None, None, None, None, None, None, 0) == -1
    assert lib.gjkepa_hull_batch_device(0, None, None, None, 1, None, None, None, None, None, None, None, None) == -1
    assert lib.gjkepa_hull_batch_device(0, None, None, None, 0, None, None, None, None, None, None, None, None) == 0
    # a cloud whose face block does not fit the face buffer is rejected on the host
    pool = gjkepa.synth_clouds(1, 2, 8, 8, 0, dtype=np.float64)
    foff = np.array([0, 4], np.int64)   # overlapping: cloud 0 needs 12 slots
    with pytest.raises(gjkepa.GjkEpaError):
        args = [np.zeros(40, np.int32) for _ in range(3)]
        rc = lib.gjkepa_hull_batch(1, pool.verts.ctypes.data, pool.verts.size, pool.cloud_off.ctypes.data,
                                   pool.cloud_cnt.ctypes.data, 2, foff.ctypes.data, 16, args[0].ctypes.data,
                                   args[1].ctypes.data, args[2].ctypes.data, np.zeros(2, np.int8).ctypes.data,
                                   None, None, 0)
        gjkepa._check(rc, "gjkepa_hull_batch")


def test_synth_clouds_deterministic_and_shardable():
    a = gjkepa.synth_clouds(5, 100, 4, 256, 0)
    b = gjkepa.synth_clouds(5, 100, 4, 256, 0)
    assert np.array_equal(a.verts, b.verts) and np.array_equal(a.cloud_cnt, b.cloud_cnt)
    tail = gjkepa.synth_clouds(5, 30, 4, 256, 0, first_cloud=70)
    for k in range(30):
        assert np.array_equal(a.cloud(70 + k), tail.cloud(k))
    s = gjkepa.synth_clouds(5, 50, 32, 32, 1)
    assert np.allclose(np.linalg.norm(s.cloud(3), axis=1), 1, atol=1e-6)
    assert np.all(np.linalg.norm(a.cloud(3), axis=1) <= 1 + 1e-6)
    assert a.cloud_cnt.min() >= 4 and a.cloud_cnt.max() <= 256


def test_hull_mesh_vertices_dedupes_in_first_appearance_order():
    soup = np.array([[[0, 0, 0], [1, 0, 0], [0, 1, 0]], [[0, 0, 0], [0, 1, 0], [0, 0, 1]]], float)
    v = gjkepa.hull_mesh_vertices(soup)
    np.testing.assert_array_equal(v, [[0, 0, 0], [1, 0, 0], [0, 1, 0], [0, 0, 1]])


# ---------------------------------------------------------------- GPU: HIP kernels vs oracle
def assert_same(g, r, pool, what=""):
    for k in ("n_faces", "n_verts", "status"):
        np.testing.assert_array_equal(g[k], r[k], err_msg=f"{what} {k}")
    for c in range(pool.n_clouds):
        fg, vg = per_cloud(g, pool, c)
        fr, vr = per_cloud(r, pool, c)
        assert np.array_equal(fg, fr), (what, "faces", c)
        assert np.array_equal(vg, vr), (what, "vert_idx", c)
        o, nv = int(pool.cloud_off[c]), int(r["n_verts"][c])
        assert np.array_equal(g["hull_verts"][o:o + 3 * nv], r["hull_verts"][o:o + 3 * nv]), (what, "hull", c)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_hull_fixture_on_gpu(orc, dtype):
    z, pool = fixture()
    pool = gjkepa.CloudPool(pool.verts.astype(dtype), pool.cloud_off, pool.cloud_cnt)
    g = gjkepa.hull_batch(pool)
    r = orc.hull_batch(pool.verts, pool.cloud_off, pool.cloud_cnt)
    assert_same(g, r, pool, str(np.dtype(dtype)))
    for k in ("n_faces", "n_verts", "status"):
        np.testing.assert_array_equal(g[k], z[k])


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [0, 1])
@pytest.mark.parametrize("lo,hi", [(4, 64), (65, 256), (4, 256)])
def test_hull_random_clouds_bitexact(orc, shape, lo, hi):
    pool = gjkepa.synth_clouds(0x6A4B5C1D + shape, 1500, lo, hi, shape)
    g = gjkepa.hull_batch(pool)
    r = orc.hull_batch(pool.verts, pool.cloud_off, pool.cloud_cnt)
    assert np.all(r["status"] == OK)
    assert_same(g, r, pool, f"shape{shape} {lo}-{hi}")


@pytest.mark.gpu
def test_hull_device_api_with_torch_stream(orc):
    import torch
    pool = gjkepa.synth_clouds(11, 3000, 4, 256, 0)
    dev = torch.device("cuda", 0)
    foff = gjkepa.hull_face_offsets(pool.cloud_cnt)
    nslots = int(foff[-1] + 2 * int(pool.cloud_cnt[-1]) - 4)
    t = {k: torch.from_numpy(v).to(dev) for k, v in
         dict(p=pool.verts, off=pool.cloud_off, cnt=pool.cloud_cnt, foff=foff).items()}
    faces = torch.full((nslots, 3), -1, dtype=torch.int32, device=dev)
    nf = torch.zeros(pool.n_clouds, dtype=torch.int32, device=dev)
    nv = torch.zeros_like(nf)
    st = torch.zeros(pool.n_clouds, dtype=torch.int8, device=dev)
    hv = torch.zeros_like(t["p"])
    vi = torch.full((pool.verts.size,), -1, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        gjkepa.hull_batch_device(gjkepa.DTYPE_F32, t["p"].data_ptr(), t["off"].data_ptr(), t["cnt"].data_ptr(),
                                 pool.n_clouds, t["foff"].data_ptr(), faces.data_ptr(), nf.data_ptr(), nv.data_ptr(),
                                 st.data_ptr(), hv.data_ptr(), vi.data_ptr(), s.cuda_stream)
    s.synchronize()
    g = dict(faces=faces.cpu().numpy(), face_off=foff, n_faces=nf.cpu().numpy(), n_verts=nv.cpu().numpy(),
             status=st.cpu().numpy(), hull_verts=hv.cpu().numpy(), vert_idx=vi.cpu().numpy())
    r = orc.hull_batch(pool.verts, pool.cloud_off, pool.cloud_cnt)
    assert_same(g, r, pool, "device api")


@pytest.mark.gpu
def test_quickhull_single_cloud_api():
    cube = np.array([[x, y, z] for z in (0, 1) for y in (0, 1) for x in (0, 1)], float)
    poly, info = gjkepa.quickhull(np.r_[cube, [[0.5, 0.5, 0.5]]])
    assert info == OK and poly.shape == (12, 3, 3)
    v = gjkepa.hull_mesh_vertices(poly)
    assert len(v) == 8 and {tuple(x) for x in v} == {tuple(x) for x in cube}
    _, info = gjkepa.quickhull(np.c_[np.random.default_rng(0).normal(size=(9, 2)), np.zeros(9)])
    assert info == DEGENERATE


@pytest.mark.gpu
def test_raw_clouds_to_hulls_to_narrow_phase():
    """The caller workflow f1 enables: reduce raw clouds to hull vertices on the device, then run
    GJK/EPA on the hulls.  Interior points never win a support mapping, so hit flag, depth and
    normal are identical to running on the raw clouds (contact points may differ: the reference's
    contact-point rules look at every point within 0.1 of the support plane, :471-472, :792)."""
    n = 2000
    clouds = gjkepa.synth_clouds(21, 2 * n, 24, 96, 0, dtype=np.float64)
    rng = np.random.default_rng(4)
    shift = rng.normal(size=(n, 3)) * 1.2
    raw = [clouds.cloud(2 * k) for k in range(n)], [clouds.cloud(2 * k + 1) + shift[k] for k in range(n)]
    rawpool = gjkepa.HullPool.from_pairs(list(zip(*raw)))
    cp = gjkepa.CloudPool(rawpool.verts, rawpool.hull_off, rawpool.hull_cnt)
    h = gjkepa.hull_batch(cp)
    assert np.all(h["status"] == OK)
    hullpool = gjkepa.HullPool(h["hull_verts"], rawpool.hull_off, h["n_verts"], rawpool.pairs)
    assert h["n_verts"].sum() < 0.8 * rawpool.hull_cnt.sum()
    a = gjkepa.gjkepa_batch(rawpool, 2, 1.0)
    b = gjkepa.gjkepa_batch(hullpool, 2, 1.0)
    assert 0.1 < a["collision"].mean() < 0.95
    np.testing.assert_array_equal(a["collision"], b["collision"])
    np.testing.assert_array_equal(a["penetration_depth"], b["penetration_depth"])
    np.testing.assert_array_equal(a["collision_normal"], b["collision_normal"])
