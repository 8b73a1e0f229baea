"""Contact-list compaction: the dense, order-preserving list of hit
pairs (GJKEPA's collision_ flag, GCLIB_GJKEPA.f90:47) and their records, built on the device from
a batch's records.  Checked against numpy on the oracle's records (bit-exact: it is index and byte
work), for both record layouts, at sizes that cross tile boundaries, and on the full C2 batch."""
import numpy as np
import pytest

import gjkepa


def test_compact_api_validation_without_gpu(lib):
    assert lib.gjkepa_compact_workspace_bytes(-1) < 0
    assert lib.gjkepa_compact_hits_device(5, None, 10, None, None, None, None, 0, None) == -1
    assert lib.gjkepa_compact_hits_device(1, None, 10, None, None, None, None, 0, None) == -1   # null n_hits


def run_compact(recs, precision, with_records=True):
    import torch
    dev = torch.device("cuda", 0)
    n = len(recs)
    r = torch.from_numpy(np.frombuffer(recs.tobytes(), np.uint8).copy()).to(dev)
    idx = torch.full((max(n, 1),), -1, dtype=torch.int32, device=dev)
    hits = torch.zeros_like(r) if with_records else None
    nh = torch.full((1,), -1, dtype=torch.int64, device=dev)
    wsb = gjkepa.compact_workspace_bytes(n)
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        gjkepa.compact_hits_device(precision, r.data_ptr(), n, idx.data_ptr(), hits.data_ptr() if with_records else 0,
                                   nh.data_ptr(), ws.data_ptr(), wsb, s.cuda_stream)
    s.synchronize()
    k = int(nh.item())
    out = np.frombuffer(hits.cpu().numpy().tobytes(), recs.dtype)[:k] if with_records else None
    return idx.cpu().numpy()[:k], out, k


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 255, 4096, 4097, 50000])
@pytest.mark.parametrize("precision", [gjkepa.PREC_F64, gjkepa.PREC_F32])
def test_compaction_matches_numpy(n, precision):
    pool = gjkepa.synth_pairs(31, n, 16, 32, 2.5)
    recs = gjkepa.gjkepa_batch(pool, 2, 1.0, precision=precision)
    idx, hits, k = run_compact(recs, precision)
    want = np.nonzero(recs["collision"] != 0)[0]
    assert k == len(want)
    np.testing.assert_array_equal(idx, want)
    assert hits.tobytes() == recs[want].tobytes()
    idx2, _, k2 = run_compact(recs, precision, with_records=False)
    assert k2 == k and np.array_equal(idx2, want)


@pytest.mark.gpu
def test_compaction_full_c2_batch(orc):
    pool = gjkepa.synth_pairs(0x6A4B5C1D, 1 << 20, 32, 32, 2.5)
    recs = gjkepa.gjkepa_batch(pool, 2, 1.0)
    idx, hits, k = run_compact(recs, gjkepa.PREC_F64)
    want = np.nonzero(recs["collision"] != 0)[0]
    assert 0.7 < k / len(recs) < 0.75
    assert np.array_equal(idx, want) and hits.tobytes() == recs[want].tobytes()
    sub = want[:2000]
    ref = orc.gjkepa_batch(gjkepa.HullPool(pool.verts, pool.hull_off, pool.hull_cnt, pool.pairs[sub]), 2, 1.0)
    assert hits[:2000].tobytes() == ref.tobytes()
