"""N>1 path on CPU: world_size-2 gloo.  Each rank generates its contiguous shard of one logical job
(shard.shard_range + gjkepa_synth_pairs(first_pair)), computes its contact records (oracle: the CPU
checker stands in for the kernels here) and the ranks all-gather the records exactly as bench.py
does with RCCL on MI355X.  The gathered bytes must equal a single-process run of the whole job."""
import os
import socket
import sys

import numpy as np
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
