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
