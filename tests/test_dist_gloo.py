"""N>1 path on CPU: world_size-2 gloo.  Each rank takes its contiguous shard of one logical job
(the library's gjkepa_shard_range + gjkepa_synth_pairs(first_pair)), computes its contact records
(oracle: the CPU checker stands in for the kernels here) and the ranks all-gather the records in
rank order, as bench.py does with the library's RCCL communicator on MI355X.  The gathered bytes must
equal a single-process run of the whole job."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOTAL = 512


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    sys.path[:0] = [os.path.join(ROOT, "collision-detect-gjk-epa_amd"), os.path.join(ROOT, "oracle")]
    import torch.distributed as dist

    import gjkepa
    import oracle
    import shard

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    first, count = shard.shard_range(TOTAL, world, rank)
    pool = gjkepa.synth_pairs(0x6A4B5C1D, count, 32, 32, 2.5, first_pair=first)
    recs = oracle.gjkepa_batch(pool, 2, 1.0, nthreads=2)
    local = torch.from_numpy(recs.view(np.uint8).reshape(-1).copy())
    full = shard.allgather_records(local, world)
    if rank == 0:
        np.save(os.path.join(outdir, "gathered.npy"), full.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_allgather_matches_single_process(tmp_path, orc):
    import gjkepa

    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    gathered = np.load(tmp_path / "gathered.npy")
    whole = gjkepa.synth_pairs(0x6A4B5C1D, TOTAL, 32, 32, 2.5)
    ref = orc.gjkepa_batch(whole, 2, 1.0)
    assert gathered.tobytes() == ref.view(np.uint8).reshape(-1).tobytes()


def _exchange_worker(rank, world, port, outdir):
    sys.path[:0] = [os.path.join(ROOT, "collision-detect-gjk-epa_amd")]
    import torch.distributed as dist

    import gjkepa
    import shard

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    ex = shard.RecordExchange(1024, world, rank, "cpu", gjkepa.PREC_F64)    # gloo: host-staged, in line
    for step in range(7):                    # what bench.py does per step: fill a buffer, submit it
        buf = ex.buffer()
        buf.fill_(16 * rank + step)
        ex.submit()
    ex.drain()
    if rank == 0:
        np.save(os.path.join(outdir, "last.npy"), ex.last_gathered.numpy())
        np.save(os.path.join(outdir, "nbuf.npy"), np.array([len(ex.local)]))
    dist.barrier()
    dist.destroy_process_group()


def test_record_exchange_host_staged(tmp_path):
    """shard.RecordExchange, the per-step all-gather bench.py runs for N > 1, in its gloo rehearsal
    mode: every rank ends with every rank's last-step records, in rank order, and a rank's buffer is
    its own slot of the gathered buffer (the RCCL mode gathers in place)."""
    world = 2
    mp.spawn(_exchange_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    last = np.load(tmp_path / "last.npy")
    want = np.concatenate([np.full(1024, 16 * r + 6, np.uint8) for r in range(world)])
    assert np.array_equal(last, want)
    assert int(np.load(tmp_path / "nbuf.npy")[0]) == 1


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_library_shard_range_tiles_the_job(world):
    """gjkepa_shard_range (C-ABI, host-only): contiguous shards in rank order that tile [0, n) exactly,
    sizes differing by at most one — the split gjkepa_batch_multi and bench.py use."""
    import gjkepa

    for n in (0, 1, 7, 1 << 21, (1 << 24) + 5):
        nxt = 0
        sizes = []
        for r in range(world):
            first, count = gjkepa.shard_range(n, world, r)
            assert first == nxt
            nxt += count
            sizes.append(count)
        assert nxt == n and max(sizes) - min(sizes) <= 1
    with pytest.raises(gjkepa.GjkEpaError):
        gjkepa.shard_range(10, world, world)


def test_multi_device_argument_checks():
    """gjkepa_batch_multi rejects an empty device list and a pool that one gjkepa_batch call would
    reject (a pair naming a missing hull, a hull outside the vertex pool) before touching any device."""
    import gjkepa

    pool = gjkepa.synth_pairs(0x6A4B5C1D, 4, 8, 8, 2.5)
    with pytest.raises(gjkepa.GjkEpaError, match="device list"):
        gjkepa.gjkepa_batch_multi(pool, [])
    bad_pair = gjkepa.HullPool(pool.verts, pool.hull_off, pool.hull_cnt, pool.pairs.copy())
    bad_pair.pairs[3, 1] = len(pool.hull_cnt)
    with pytest.raises(gjkepa.GjkEpaError, match="missing hull"):
        gjkepa.gjkepa_batch_multi(bad_pair, [0, 0])
    for off in (-3, len(pool.verts) - 3 * int(pool.hull_cnt[5]) + 1):   # 1-based slip / past the end
        o = pool.hull_off.copy()
        o[5] = off
        with pytest.raises(gjkepa.GjkEpaError, match="outside the vertex pool"):
            gjkepa.gjkepa_batch_multi(gjkepa.HullPool(pool.verts, o, pool.hull_cnt, pool.pairs), [0, 0, 0])
