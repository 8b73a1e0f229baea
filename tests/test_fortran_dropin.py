"""The Fortran drop-in: a caller written against the reference interface (USE GCLIB_GJKEPA;
CALL GJKEPA(...)) runs unchanged on the MI355X path.  tests/fortran/test_dropin.f90 prints every
query; each line is compared with the oracle bit for bit."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "fortran", "build", "test_dropin")
CUBE = np.array([[x, y, z] for z in (0, 1) for y in (0, 1) for x in (0, 1)], float)
OFFS = [(0.5, 0.2, 0.1), (1, 0, 0), (1 + 1e-9, 0, 0), (0, 0, 1e-3), (0.5, 0.5, 0.1), (0.3, 0.2, 0.1),
        (0.9, 0.8, 0.7), (0.9, 0.25, 0), (3, 0, 0), (0, 0, 0), (0.3, 0.3, 0.3), (1, 1, 1)]


def test_driver_built():
    assert os.path.exists(EXE), "run __graft_entry__.build()"


@pytest.mark.gpu
def test_fortran_gjkepa_matches_oracle(orc):
    out = subprocess.run([EXE], capture_output=True, text=True, timeout=300, env=dict(os.environ, OMP_NUM_THREADS="4"))
    assert out.returncode == 0, out.stderr
    lines = [ln.split() for ln in out.stdout.splitlines() if ln[:1] in ("Q", "B")]
    assert len(lines) == 48
    for f in lines:
        v, i = int(f[1]), int(f[2])
        hit, typ, st = f[3] == "T", int(f[4]), int(f[5])
        vals = np.array([float(x) for x in f[6:]])
        r = orc.gjkepa(v, 1e-3, CUBE, CUBE + np.asarray(OFFS[i - 1]))
        want = np.concatenate([[r["penetration_depth"]], r["collision_normal"], r["collision_point"], r["nearest_points"]])
        assert hit == bool(r["collision"]) and typ == r["colli_type"] and st == r["status"], f
        both_nan = np.isnan(vals) & np.isnan(want)
        assert np.all((vals == want) | both_nan), (f, want)
    mism = [ln for ln in out.stdout.splitlines() if ln.startswith("OMP_MISMATCH")]
    assert mism and int(mism[0].split()[1]) == 0, "OpenMP callers disagree with the batched entry"
    mm = [ln for ln in out.stdout.splitlines() if ln.startswith("MULTI_MISMATCH")]
    assert mm and int(mm[0].split()[1]) == 0, "GJKEPA_BATCH(devices_=...) disagrees with the one-device entry"


QH_EXE = os.path.join(ROOT, "tests", "fortran", "build", "test_quickhull")


def test_quickhull_driver_built():
    assert os.path.exists(QH_EXE), "run __graft_entry__.build()"


@pytest.mark.gpu
def test_fortran_quickhull_matches_oracle(orc, tmp_path):
    """USE GCLIB_QuickHull / GCLIB_DeHull; CALL QuickHull(points, polytope, info) and
    getHullMeshesVertex(polytope, points, info) with the reference's call-site argument lists
    (GCLIB_GJKEPA.f90:920, :950), plus QUICKHULL_BATCH, against the oracle hull."""
    import gjkepa
    rng = np.random.default_rng(8)
    clouds = [np.r_[CUBE, [[0.5, 0.5, 0.5]]], rng.normal(size=(40, 3)), rng.uniform(-1, 1, (200, 3)),
              np.c_[rng.normal(size=(12, 2)), np.zeros(12)], rng.normal(size=(3, 3))]
    clouds = [np.asarray(c, np.float32).astype(np.float64) for c in clouds]
    path = tmp_path / "clouds.txt"
    with open(path, "w") as fh:
        fh.write(f"{len(clouds)}\n")
        for c in clouds:
            fh.write(f"{len(c)}\n" + "".join(f"{x:.17g} {y:.17g} {z:.17g}\n" for x, y, z in c))
    out = subprocess.run([QH_EXE, str(path)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    pool = gjkepa.CloudPool.from_list(clouds)
    r = orc.hull_batch(pool.verts, pool.cloud_off, pool.cloud_cnt)
    lines = out.stdout.splitlines()
    q = [i for i, ln in enumerate(lines) if ln.startswith("Q ")]
    b = [ln.split() for ln in lines if ln.startswith("B ")]
    assert len(q) == len(clouds) == len(b)
    for c, i in enumerate(q):
        _, _, info, nf, nv = lines[i].split()
        assert int(info) == r["status"][c] and int(nf) == r["n_faces"][c] and int(nv) == r["n_verts"][c]
        fo = r["face_off"][c]
        want = clouds[c][r["faces"][fo:fo + r["n_faces"][c]]].reshape(-1, 9)
        got = np.array([[float(x) for x in lines[i + 1 + f].split()[1:]] for f in range(int(nf))]).reshape(-1, 9)
        np.testing.assert_array_equal(got, want)
        st, nfb, nvb = int(b[c][2]), int(b[c][3]), int(b[c][4])
        assert (st, nfb, nvb) == (r["status"][c], r["n_faces"][c], r["n_verts"][c])
        tri = np.array([int(x) for x in b[c][5:]]).reshape(-1, 3) - 1
        np.testing.assert_array_equal(tri, r["faces"][fo:fo + nfb])


BP_EXE = os.path.join(ROOT, "tests", "fortran", "build", "test_broadphase")


def test_broadphase_driver_built():
    assert os.path.exists(BP_EXE), "run __graft_entry__.build()"


@pytest.mark.gpu
def test_fortran_broadphase_matches_oracle(orc, tmp_path):
    """USE GCLIB_GJKEPA; CALL GJKEPA_BROADPHASE(...): the reference sphere test's pair list for a
    pooled hull set, 1-based and ascending, identical to the oracle's."""
    import gjkepa
    pool = gjkepa.synth_scene(77, 400, 8, 40, 12.0, dtype=np.float64)
    path = tmp_path / "hulls.txt"
    with open(path, "w") as fh:
        fh.write(f"{pool.hull_cnt.size}\n")
        for h in range(pool.hull_cnt.size):
            p = pool.hull(h)
            fh.write(f"{len(p)}\n" + "".join(f"{x:.17g} {y:.17g} {z:.17g}\n" for x, y, z in p))
    out = subprocess.run([BP_EXE, str(path)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.splitlines()
    n, info = (int(x) for x in lines[0].split()[1:])
    got = np.array([[int(x) for x in ln.split()[1:]] for ln in lines[1:] if ln.startswith("P")]).reshape(-1, 2) - 1
    want, m = orc.broadphase(pool.verts, pool.hull_off, pool.hull_cnt)
    assert info == 0 and n == m > 0
    np.testing.assert_array_equal(got, want)


CL_EXE = os.path.join(ROOT, "tests", "fortran", "build", "test_collide")


def test_collide_driver_built():
    assert os.path.exists(CL_EXE), "run __graft_entry__.build()"


@pytest.mark.gpu
def test_fortran_collide_matches_oracle(orc, tmp_path):
    """USE GCLIB_GJKEPA; CALL GJKEPA_COLLIDE(...): the caller's all-pairs GJKEPA loop in one call —
    the colliding pairs (1-based, ascending) with GJKEPA's outputs, equal to the oracle's broad
    phase + GJKEPA on each candidate (reals printed with 17 significant digits: exact)."""
    import gjkepa
    pool = gjkepa.synth_scene(78, 300, 8, 40, 10.0, dtype=np.float64)
    path = tmp_path / "hulls.txt"
    with open(path, "w") as fh:
        fh.write(f"{pool.hull_cnt.size}\n")
        for h in range(pool.hull_cnt.size):
            p = pool.hull(h)
            fh.write(f"{len(p)}\n" + "".join(f"{x:.17g} {y:.17g} {z:.17g}\n" for x, y, z in p))
    out = subprocess.run([CL_EXE, str(path)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.splitlines()
    n, info = (int(x) for x in lines[0].split()[1:])
    rows = [ln.split()[1:] for ln in lines[1:] if ln.startswith("C")]
    cand, _ = orc.broadphase(pool.verts, pool.hull_off, pool.hull_cnt)
    cand = cand.reshape(-1, 2)
    sub = gjkepa.HullPool(pool.verts, pool.hull_off, pool.hull_cnt, np.ascontiguousarray(cand.reshape(-1)))
    recs = orc.gjkepa_batch(sub, 2, 1.0)
    hit = recs["collision"] != 0
    assert info == 0 and n == int(hit.sum()) == len(rows) > 0
    got_pairs = np.array([[int(r[0]), int(r[1])] for r in rows]) - 1
    np.testing.assert_array_equal(got_pairs, cand[hit])
    want = recs[hit]
    for r, w in zip(rows, want):
        assert int(r[2]) == w["colli_type"] and int(r[3]) == w["status"]
        vals = np.array([float(x) for x in r[4:]])
        ref = np.concatenate([[w["penetration_depth"]], w["collision_normal"], w["collision_point"]])
        np.testing.assert_array_equal(vals, ref)
