"""gjkepa_batch_device is graph-capturable (include/gjkepa.h): the whole launch chain — counter reset,
the tier kernels and (for batches of 64K pairs and up) the contact passes forked onto the library's
second stream and joined back — captured into a HIP graph and replayed gives the records of a
direct call, byte for byte, replay after replay."""
import os

import numpy as np
import pytest

import gjkepa

pytestmark = pytest.mark.gpu


REPLAYS = int(os.environ.get("GJKEPA_GRAPH_REPLAYS", "10"))


def _guard_report():
    """Argument-guard report of a GJKEPA_DIAG_GUARD build (tools/build_variant.sh guard), else None."""
    import ctypes
    lib = gjkepa.load()
    if not hasattr(lib, "gjkepa_diag_guard"):
        return None
    out = (ctypes.c_uint32 * 8)()
    assert lib.gjkepa_diag_guard(out, 1) == 8
    return list(out)


@pytest.mark.parametrize("lo,hi,rmax,n", [(32, 32, 2.5, 3000), (8, 256, 2.5, 3000), (32, 32, 2.5, 70000)])
@pytest.mark.parametrize("prec", [gjkepa.PREC_F32, gjkepa.PREC_F64], ids=["f32", "f64"])
def test_captured_chain_replays_bitexact(lo, hi, rmax, n, prec):
    import torch
    dev = torch.device("cuda", 0)
    pool = gjkepa.synth_pairs(0x5EED, n, lo, hi, rmax, dtype=np.float32)
    verts = torch.from_numpy(pool.verts).to(dev)
    off = torch.from_numpy(pool.hull_off).to(dev)
    cnt = torch.from_numpy(pool.hull_cnt).to(dev)
    prs = torch.from_numpy(pool.pairs.reshape(-1)).to(dev)
    wsb = gjkepa.workspace_bytes(n)
    ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)

    def run(out, stream):
        gjkepa.gjkepa_batch_device(2, 1.0, gjkepa.DTYPE_F32, prec, verts.data_ptr(), off.data_ptr(),
                                   cnt.data_ptr(), prs.data_ptr(), n, out.data_ptr(), ws.data_ptr(), wsb, stream)

    work = torch.cuda.Stream(dev)
    ref = torch.zeros(n * (128 if prec == gjkepa.PREC_F64 else 64), dtype=torch.uint8, device=dev)
    out = torch.zeros_like(ref)
    for name, t in (("verts", verts), ("off", off), ("cnt", cnt), ("pairs", prs), ("ws", ws), ("ref", ref), ("out", out)):
        print(f"graph-test buffer {name}: {t.data_ptr():#x} + {t.numel() * t.element_size()} B", flush=True)
    torch.cuda.synchronize(dev)
    with torch.cuda.stream(work):
        run(ref, work.cuda_stream)
    torch.cuda.synchronize(dev)
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream(dev)
    with torch.cuda.graph(g, stream=side):
        run(out, side.cuda_stream)
    torch.cuda.synchronize(dev)
    for i in range(REPLAYS):
        print(f"graph-test replay {i}", flush=True)
        with torch.cuda.stream(work):
            out.zero_()
            g.replay()
        torch.cuda.synchronize(dev)
        rep = _guard_report()
        if rep is not None:
            print(f"graph-test guard after replay {i}: {rep}", flush=True)
            assert rep[0] == 0, f"kernel argument block changed after enqueue: {rep}"
        assert torch.equal(out, ref)
    # a direct call after the replays still matches (the graph left no state behind)
    with torch.cuda.stream(work):
        out.zero_()
        run(out, work.cuda_stream)
    torch.cuda.synchronize(dev)
    assert torch.equal(out, ref)
    expect = gjkepa.gjkepa_batch(pool, 2, 1.0, precision=prec)
    assert ref.cpu().numpy().tobytes() == expect.tobytes()
    del g
