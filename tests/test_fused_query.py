"""The one-kernel query path (query_kernel: GJK, EPA and the contact features in one wave per pair)
that serves batches of up to GJKEPA_FUSED_MAX (64) pairs, e.g. combined single-pair gjkepa_query
calls.  It runs the tier kernels' device functions with the largest tier's capacities, so every
record must equal the tier chain's and the oracle's byte for byte: each golden fixture and the
branch-coverage fixture (the reference's rare paths, incl. DEGENERATE, EPA_MAXITER, BAD_VERSION,
BAD_INPUT) are run in 64-pair batches and compared with their committed oracle records."""
import os

import numpy as np
import pytest

import gjkepa

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FUSED_MAX = 64


def _chunked(pool, version, tol, size=FUSED_MAX):
    out = []
    for i in range(0, pool.n_pairs, size):
        sub = gjkepa.HullPool(pool.verts, pool.hull_off, pool.hull_cnt, pool.pairs[i:i + size])
        out.append(gjkepa.gjkepa_batch(sub, version, tol))
    return np.concatenate(out)


@pytest.mark.parametrize("name,versions", [("c1_cubes", (1, 2, 3)), ("c2_32v", (1, 2, 3)), ("c4_mixed", (1, 2, 3)),
                                           ("c5_deep", (2,)), ("branch_cov", (1, 2, 3, 4))])
def test_fused_batches_bitexact(name, versions):
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    pool = gjkepa.HullPool(z["verts"], z["hull_off"], z["hull_cnt"], z["pairs"])
    tol = float(z["tol_ff"]) if "tol_ff" in z.files else 1.0
    n = min(pool.n_pairs, 1024)
    pool = gjkepa.HullPool(pool.verts, pool.hull_off, pool.hull_cnt, pool.pairs[:n])
    for v in versions:
        g = _chunked(pool, v, tol)
        ref = z[f"rec_v{v}"].reshape(-1).view(gjkepa.REC64)[:n]
        same = (g.view(np.uint8).reshape(n, -1) == ref.view(np.uint8).reshape(n, -1)).all(axis=1)
        assert same.all(), (name, v, np.nonzero(~same)[0][:10])


def test_fused_fp32_compute_agrees_with_chain():
    """fp32 compute: the fused path and the tier chain run the same arithmetic, so they agree bit for bit."""
    pool = gjkepa.synth_pairs(0xF00D, 4 * FUSED_MAX, 8, 256, 2.5, dtype=np.float32)
    fused = _chunked(pool, 2, 1.0)
    fused32 = np.concatenate([gjkepa.gjkepa_batch(gjkepa.HullPool(pool.verts, pool.hull_off, pool.hull_cnt,
                                                                    pool.pairs[i:i + FUSED_MAX]), 2, 1.0,
                                                  precision=gjkepa.PREC_F32)
                              for i in range(0, pool.n_pairs, FUSED_MAX)])
    chain = gjkepa.gjkepa_batch(pool, 2, 1.0)                                  # 256 pairs: the tier chain
    chain32 = gjkepa.gjkepa_batch(pool, 2, 1.0, precision=gjkepa.PREC_F32)
    assert fused.tobytes() == chain.tobytes()
    assert fused32.tobytes() == chain32.tobytes()
