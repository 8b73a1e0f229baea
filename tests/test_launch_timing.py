"""Per-launch timing of the tier chain (include/gjkepa.h gjkepa_launch_timing), the basis of bench.py's
dominant-kernel roofline: every launch of an overlapped chain is reported once, on the stream it ran
on, with start <= end inside the chain (launches of one stream in order); timing never changes a
record, and the records match the oracle."""
import numpy as np
import pytest

import gjkepa

pytestmark = pytest.mark.gpu
SEED = 0x6A4B5C1D


def _device_run(pool, timing: bool):
    import torch
    dev = torch.device("cuda", 0)
    v = torch.from_numpy(pool.verts).to(dev)
    o = torch.from_numpy(pool.hull_off).to(dev)
    c = torch.from_numpy(pool.hull_cnt).to(dev)
    p = torch.from_numpy(pool.pairs.reshape(-1).copy()).to(dev)
    n = pool.n_pairs
    out = torch.zeros(n * 128, dtype=torch.uint8, device=dev)
    wsb = gjkepa.workspace_bytes_for(n, gjkepa.large_pairs(pool))
    ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream(dev)
    gjkepa.launch_timing(timing)
    for _ in range(2):
        gjkepa.gjkepa_batch_device(2, 1.0, gjkepa.DTYPE_F32, gjkepa.PREC_F64, v.data_ptr(), o.data_ptr(), c.data_ptr(),
                                   p.data_ptr(), n, out.data_ptr(), ws.data_ptr(), wsb, s.cuda_stream)
    gjkepa.launch_timing(False)
    lt = gjkepa.launch_timing_read()
    torch.cuda.synchronize(dev)
    return np.frombuffer(out.cpu().numpy().tobytes(), gjkepa.REC64), lt


@pytest.mark.parametrize("lo,hi", [(32, 32), (8, 256)])
def test_launch_timing_covers_the_chain(orc, lo, hi):
    n = 70000                                         # >= 64K pairs: the overlapped (multi-stream) chain
    pool = gjkepa.synth_pairs(SEED, n, lo, hi, 2.5)
    plain, lt0 = _device_run(pool, False)
    timed, lt = _device_run(pool, True)
    assert len(lt0) == 0
    assert plain.tobytes() == timed.tobytes()
    assert sorted(set(lt["chain"].tolist())) == [0, 1]
    one = lt[lt["chain"] == 1]
    kinds = [(k.decode(), int(t)) for k, t in zip(one["kernel"], one["tier"])]
    assert kinds[0] == ("reset", 0) and kinds[1] == ("gjk", 0) and kinds[2] == ("gjk", 1)
    assert sum(1 for k in kinds if k == ("epa", 0)) == 2           # EPA tier 0 in two parts
    assert {("epa", t) for t in range(6)} <= set(kinds) and ("contact", 0) in kinds
    assert (one["start_ms"] >= 0).all() and (one["end_ms"] >= one["start_ms"]).all()
    assert one["stream"].max() >= 1                                # internal streams reported
    e0 = one[(one["kernel"] == b"epa") & (one["tier"] == 0)]
    assert e0["first_pair"][0] == 0 and e0["first_pair"][1] + e0["n_pairs"][1] == n
    e2 = one[(one["kernel"] == b"epa") & (one["tier"] == 2)]
    e3 = one[(one["kernel"] == b"epa") & (one["tier"] == 3)]
    if e2["stream"][0] == e3["stream"][0]:                          # in sequence (GJKEPA_E23_STREAMS 1)
        assert e3["start_ms"][0] >= e2["end_ms"][0]
    sub = np.arange(0, n, 7)
    ref = orc.gjkepa_batch(gjkepa.HullPool(pool.verts, pool.hull_off, pool.hull_cnt, pool.pairs[sub]), 2, 1.0)
    assert timed[sub].tobytes() == ref.tobytes()
