"""CPU tests of the oracle (the checker): known answers, golden fixtures, independent geometry.

The reference ships no tests or golden vectors and cannot be built here, so the
oracle is pinned by (1) the known-answer cube cases recorded from the survey's probe of the
reference, (2) scipy Qhull ground truth for depth/normal/hit, and (3) the
committed golden fixtures (regression; see tests/golden/make_golden.py).
"""
import os

import numpy as np
import pytest

import gjkepa
import parity

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CUBE = np.array([[x, y, z] for z in (0, 1) for y in (0, 1) for x in (0, 1)], float)


def q(orc, off, version=2, tol=1e-3):
    return orc.gjkepa(version, tol, CUBE, CUBE + np.asarray(off, float))


# SURVEY.md Appendix C (unit cube A, B = A + offset, TOL_FF_ = 1e-3)
@pytest.mark.parametrize("version", [1, 2])
def test_c1_cube_baseline(orc, version):
    r = q(orc, (0.5, 0.2, 0.1), version)
    assert r["collision"] == 1 and r["colli_type"] == 2 and r["status"] == 0
    assert r["penetration_depth"] == pytest.approx(0.5, abs=1e-14)
    assert np.allclose(r["collision_normal"], [1, 0, 0], atol=1e-14)
    assert np.allclose(r["collision_point"], [1, 0.5, 0.5], atol=1e-14)
    assert np.allclose(r["nearest_points"][:3], [1, 0, 0])


def test_c1_cube_version3(orc):
    r = q(orc, (0.5, 0.2, 0.1), 3)
    assert np.allclose(r["collision_point"], [0.5, 1.2, 0.5], atol=1e-14)
    assert np.allclose(r["collision_normal"], [1, 0, 0], atol=1e-14)


@pytest.mark.parametrize("off,depth,normal", [
    ((0.5, 0.5, 0.1), 0.5, (0, 1, 0)),      # exact x/y tie resolved by path order
    ((0.3, 0.2, 0.1), 0.7, (1, 0, 0)),
    ((0.9, 0.8, 0.7), 0.1, (1, 0, 0)),
    ((0.9, 0.25, 0.0), 0.1, (1, 0, 0)),
    ((0.0, 0.0, 1e-3), 0.999, (0, 0, 1)),
])
def test_known_answers(orc, off, depth, normal):
    r = q(orc, off)
    assert r["collision"] == 1 and r["status"] == 0
    assert r["penetration_depth"] == pytest.approx(depth, abs=1e-12)
    assert np.allclose(r["collision_normal"], normal, atol=1e-12)


def test_exact_touch_counts_as_hit(orc):
    # Appendix C: (1,0,0) touching is a hit with depth 0.  The probe's normal sign (-x) came from
    # its stand-in hull's face winding (origin on the face, dot = 0: no re-orientation); the
    # re-supplied hull winds faces outward, giving +x (from hull 1 towards hull 2).  Unpinned tie.
    r = q(orc, (1, 0, 0))
    assert r["collision"] == 1 and r["status"] == 0 and r["penetration_depth"] == 0.0
    assert abs(abs(r["collision_normal"][0]) - 1) < 1e-12


def test_misses(orc):
    for off in [(1 + 1e-9, 0, 0), (3, 0, 0)]:
        r = q(orc, off)
        assert r["collision"] == 0 and r["colli_type"] == 0 and r["status"] == 0
        assert r["penetration_depth"] == 0 and not np.any(r["collision_normal"])


def test_version3_normal_projection_nan(orc):
    r = q(orc, (0, 0, 1e-3), 3)
    assert np.all(np.isnan(r["collision_normal"])) and r["colli_type"] == 1


@pytest.mark.parametrize("off", [(0, 0, 0), (0.3, 0.3, 0.3), (1, 1, 1)])
def test_reference_abort_cases_are_degenerate(orc, off):
    # the reference STOPs in DIST_PF_SIGN (GCLIB_GJKEPA.f90:1369-1373); here: status DEGENERATE
    r = q(orc, off)
    assert r["status"] == gjkepa.STATUS_DEGENERATE and r["collision"] == 1
    assert r["penetration_depth"] == 0


def test_bad_version_only_on_hits(orc):
    assert q(orc, (0.5, 0.2, 0.1), 7)["status"] == gjkepa.STATUS_BAD_VERSION
    assert q(orc, (3, 0, 0), 7)["status"] == gjkepa.STATUS_OK     # misses never reach EPA_solu


def test_bad_input(orc):
    r = orc.gjkepa(2, 1.0, np.zeros((0, 3)), CUBE)
    assert r["status"] == gjkepa.STATUS_BAD_INPUT


@pytest.mark.parametrize("name", ["c1_cubes", "c2_32v", "c4_mixed", "c5_deep"])
def test_golden_fixtures(orc, name):
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    pool = gjkepa.HullPool(z["verts"], z["hull_off"], z["hull_cnt"], z["pairs"])
    for v in (1, 2, 3):
        got = orc.gjkepa_batch(pool, v, float(z["tol_ff"]))
        assert got.view(np.uint8).reshape(len(got), -1).tobytes() == z[f"rec_v{v}"].tobytes(), (name, v)


@pytest.mark.parametrize("name", ["c2_32v", "c4_mixed", "c5_deep"])
def test_oracle_vs_qhull_ground_truth(orc, name):
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    pool = gjkepa.HullPool(z["verts"], z["hull_off"], z["hull_cnt"], z["pairs"])
    r = orc.gjkepa_batch(pool, 2, 1.0)
    ok = r["status"] == 0
    hit = r["collision"] != 0
    inside = z["qhull_inside"]
    assert np.array_equal(hit[ok], inside[ok]), "hit flag disagrees with the Minkowski hull"
    m = ok & hit
    d_ref = z["qhull_depth"][m]
    assert np.all(np.abs(r["penetration_depth"][m] - d_ref) <= 1e-9 * np.maximum(1, d_ref))
    assert np.all(np.abs(r["collision_normal"][m] - z["qhull_normal"][m]) <= 1e-9)
    assert ok.mean() > 0.99


def test_parity_helper_detects_differences(orc):
    z = np.load(os.path.join(GOLDEN, "c2_32v.npz"))
    ref = z["rec_v2"].copy().view(gjkepa.REC64).reshape(-1)
    mod = ref.copy()
    assert parity.compare(mod, ref)["ok"]
    mod["penetration_depth"][np.nonzero(ref["collision"])[0][0]] *= 1 + 1e-5
    assert not parity.compare(mod, ref)["ok"]
    mod = ref.copy()
    mod["collision"][0] ^= 1
    assert parity.compare(mod, ref)["hit_mismatch"] == 1
