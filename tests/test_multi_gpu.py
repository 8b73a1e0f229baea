"""Multi-GPU product path on the GPU (SURVEY.md §8 row e, config C3).

- C3 per-rank workload: each of two ranks owns 2^21 C2-distribution pairs at first_pair = r * 2^21
  (the library's shard rule); each shard, run through the C-ABI on the GPU, is byte-identical to the
  matching half of one contiguous 2^22-pair run and to the oracle on a subsample.
- gjkepa_batch_multi (one process, a device list) equals gjkepa_batch and the oracle.  The box has
  one GPU, so the lists repeat device 0 (2, 3 and 8 shards): every shard still goes through the
  shard / hull-range rebase / per-shard thread path, and the shards of one device run in turn.
- The library's RCCL communicator (world 1 here; the driver's 8-GPU run exercises world 8): the
  in-place and out-of-place all-gather of records returns them unchanged; shard.RecordExchange's
  overlapped, double-buffered gather over it, and over the torch.distributed "nccl" (RCCL) group that
  bench.py falls back to when the library's communicator cannot start.
- Config C3 whole: the 2^24-pair job as 8 ranks of bench.py (torch.distributed.run, one process per
  rank, all on this box's GPU, host-staged gather), then in this process the same 2^24 pairs as one
  contiguous gjkepa_batch and as gjkepa_batch_multi over 8 shards of device 0: every rank's slot of the
  gathered buffer hashes to the contiguous run's records, and a subsample of every shard matches the
  oracle.  The reference's own parallelism is its caller's OpenMP loop over GJKEPA (:9, :16).
"""
import hashlib
import json
import os
import subprocess
import sys
import time

import numpy as np
import pytest

import gjkepa

pytestmark = pytest.mark.gpu
SEED = 0x6A4B5C1D
PER_RANK = 1 << 21
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
C3_RANKS = 8
_c3: dict = {}


def _log(msg: str) -> None:
    """Progress of the long C3 tests, also into gpurun_out/ when it exists (a liveness record)."""
    print(msg, flush=True)
    d = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(d):
        with open(os.path.join(d, "c3_progress.log"), "a") as f:
            f.write(f"{time.strftime('%H:%M:%S')} {msg}\n")


def _bytes(a):
    return a.view(np.uint8).reshape(len(a), -1)


def test_c3_rank_shards_match_contiguous_run_and_oracle(orc):
    whole = gjkepa.synth_pairs(SEED, 2 * PER_RANK, 32, 32, 2.5)
    ref = gjkepa.gjkepa_batch(whole, 2, 1.0)
    for rank in range(2):
        first, count = gjkepa.shard_range(2 * PER_RANK, 2, rank)
        assert (first, count) == (rank * PER_RANK, PER_RANK)
        pool = gjkepa.synth_pairs(SEED, count, 32, 32, 2.5, first_pair=first)
        got = gjkepa.gjkepa_batch(pool, 2, 1.0)
        assert got.tobytes() == ref[first:first + count].tobytes(), rank
        sub = np.arange(0, count, 97)                      # oracle on a ~21.6k-pair subsample
        spool = gjkepa.HullPool(pool.verts, pool.hull_off, pool.hull_cnt, pool.pairs[sub])
        o = orc.gjkepa_batch(spool, 2, 1.0)
        assert got[sub].tobytes() == o.tobytes(), rank


@pytest.mark.parametrize("ndev", [1, 2, 3, 8])
@pytest.mark.parametrize("lo,hi", [(32, 32), (8, 256)])
def test_batch_multi_matches_batch(lo, hi, ndev, orc):
    """Contiguous pairs (each pair owns its hulls) in ndev shards on device 0."""
    pool = gjkepa.synth_pairs(SEED, 50001, lo, hi, 2.5)       # odd size: shards differ by one pair
    a = gjkepa.gjkepa_batch(pool, 2, 1.0)
    b = gjkepa.gjkepa_batch_multi(pool, [0] * ndev, 2, 1.0)
    assert a.tobytes() == b.tobytes()
    sub = np.arange(0, pool.n_pairs, 211)
    o = orc.gjkepa_batch(gjkepa.HullPool(pool.verts, pool.hull_off, pool.hull_cnt, pool.pairs[sub]), 2, 1.0)
    assert b[sub].tobytes() == o.tobytes()


@pytest.mark.parametrize("ndev", [1, 2, 3, 8])
def test_batch_multi_shared_hull_pool(orc, ndev):
    """A pool whose pairs share hulls out of order (a broad-phase list): every shard's hull range
    straddles the others'; each shard copies only the range it references, rebased.  Equal to one
    gjkepa_batch call and to the oracle."""
    rng = np.random.default_rng(3)
    hulls = gjkepa.synth_pairs(SEED, 300, 8, 64, 2.5)
    prs = rng.integers(0, 600, size=(4000, 2)).astype(np.int32)
    pool = gjkepa.HullPool(hulls.verts, hulls.hull_off, hulls.hull_cnt, prs)
    g = gjkepa.gjkepa_batch_multi(pool, [0] * ndev, 2, 1.0)
    assert g.tobytes() == gjkepa.gjkepa_batch(pool, 2, 1.0).tobytes()
    assert g.tobytes() == orc.gjkepa_batch(pool, 2, 1.0).tobytes()


def test_batch_multi_rejects_hull_outside_pool():
    """The whole-job argument checks of gjkepa_batch apply before sharding."""
    pool = gjkepa.synth_pairs(SEED, 64, 8, 32, 2.5)
    off = pool.hull_off.copy()
    off[7] = len(pool.verts)
    with pytest.raises(gjkepa.GjkEpaError, match="outside the vertex pool"):
        gjkepa.gjkepa_batch_multi(gjkepa.HullPool(pool.verts, off, pool.hull_cnt, pool.pairs), [0, 0])


def test_rccl_comm_world1_allgather():
    import torch

    dev = torch.device("cuda", 0)
    uid = gjkepa.Comm.unique_id()
    comm = gjkepa.Comm(1, 0, uid, 0)
    try:
        pool = gjkepa.synth_pairs(SEED, 4096, 32, 32, 2.5)
        recs = gjkepa.gjkepa_batch(pool, 2, 1.0)
        src = torch.from_numpy(_bytes(recs).reshape(-1).copy()).to(dev)
        dst = torch.zeros_like(src)
        s = torch.cuda.current_stream(dev)
        comm.allgather_records(gjkepa.PREC_F64, src.data_ptr(), dst.data_ptr(), len(recs), s.cuda_stream)
        comm.allgather_records(gjkepa.PREC_F64, src.data_ptr(), src.data_ptr(), len(recs), s.cuda_stream)  # in place
        torch.cuda.synchronize(dev)
        assert dst.cpu().numpy().tobytes() == recs.tobytes()
        assert src.cpu().numpy().tobytes() == recs.tobytes()
    finally:
        comm.close()
    assert gjkepa.Comm.backend() != "unavailable"


def test_record_exchange_rccl_overlapped_steps():
    """shard.RecordExchange's RCCL branch, the one bench.py runs at N > 1 over the library's
    communicator (world 1 here): double-buffered records, each step's all-gather on the exchange's own
    stream after that step's kernels, the next step's kernels overlapping it.  Four steps of
    gjkepa_batch_device over four different pair sets alternate between the two buffers; after each
    step `last_gathered` holds that step's records, and the other buffer still holds the previous
    step's (the compute stream waited for its gather before reusing it, and nothing wrote it early)."""
    import torch

    import shard

    dev = torch.device("cuda", 0)
    comm = gjkepa.Comm(1, 0, gjkepa.Comm.unique_id(), 0)
    try:
        n = 1 << 16
        prec = gjkepa.PREC_F64
        rb = gjkepa.load().gjkepa_record_bytes(prec)
        pools = [gjkepa.synth_pairs(SEED + 17 * s, n, 32, 32, 2.5, dtype=np.float32) for s in range(4)]
        refs = [gjkepa.gjkepa_batch(p, 2, 1.0) for p in pools]
        assert len({r.tobytes() for r in refs}) == 4
        dpools = [[torch.from_numpy(a).to(dev) for a in (p.verts, p.hull_off, p.hull_cnt, p.pairs.reshape(-1))]
                  for p in pools]
        wsb = gjkepa.workspace_bytes_for(n, max(gjkepa.large_pairs(p) for p in pools))
        ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
        ex = shard.RecordExchange(n * rb, 1, 0, dev, prec, comm=comm)
        assert ex.overlap and len(ex.gathered) == 2
        stream = torch.cuda.current_stream(dev)
        for i, (v, o, c, p) in enumerate(dpools):
            buf = ex.buffer(stream)                   # waits for the gather that last read this buffer
            assert buf.data_ptr() == ex.gathered[i % 2].data_ptr()
            gjkepa.gjkepa_batch_device(2, 1.0, gjkepa.DTYPE_F32, prec, v.data_ptr(), o.data_ptr(), c.data_ptr(),
                                       p.data_ptr(), n, buf.data_ptr(), ws.data_ptr(), wsb, stream.cuda_stream)
            ex.submit(stream)
            if i >= 1:                                 # the previous step's buffer, while this step's gather may run
                prev = ex.gathered[(i - 1) % 2].cpu().numpy().tobytes()
                assert prev == refs[i - 1].tobytes(), i
            torch.cuda.synchronize(dev)
            assert ex.last_gathered.cpu().numpy().tobytes() == refs[i].tobytes(), i
            assert ex.last.cpu().numpy().tobytes() == refs[i].tobytes(), i
        ex.drain()
        assert all(e is None for e in ex.done)
        assert ex.gathered[0].cpu().numpy().tobytes() == refs[2].tobytes()
        assert ex.gathered[1].cpu().numpy().tobytes() == refs[3].tobytes()
    finally:
        comm.close()


_TORCH_RCCL_SCRIPT = r"""
import sys, numpy as np, torch, torch.distributed as dist
sys.path.insert(0, sys.argv[1])
import gjkepa, shard
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:" + sys.argv[2], world_size=1, rank=0)
g = dist.new_group(backend="nccl")
dev = torch.device("cuda", 0)
n, prec = 1 << 15, gjkepa.PREC_F64
rb = gjkepa.load().gjkepa_record_bytes(prec)
ex = shard.RecordExchange(n * rb, 1, 0, dev, prec, comm=None, device_group=g)
assert ex.overlap and len(ex.gathered) == 2
wsb = gjkepa.workspace_bytes_for(n, 0)
ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream(dev)
for i in range(3):
    pool = gjkepa.synth_pairs(0x6A4B5C1D + 31 * i, n, 32, 32, 2.5)
    ref = gjkepa.gjkepa_batch(pool, 2, 1.0)
    v, o, c, p = (torch.from_numpy(a).to(dev) for a in (pool.verts, pool.hull_off, pool.hull_cnt, pool.pairs.reshape(-1)))
    buf = ex.buffer(st)
    gjkepa.gjkepa_batch_device(2, 1.0, gjkepa.DTYPE_F32, prec, v.data_ptr(), o.data_ptr(), c.data_ptr(), p.data_ptr(),
                               n, buf.data_ptr(), ws.data_ptr(), wsb, st.cuda_stream)
    ex.submit(st)
    torch.cuda.synchronize(dev)
    assert ex.last_gathered.cpu().numpy().tobytes() == ref.tobytes(), i
ex.drain()
dist.destroy_process_group()
print("ok")
"""


def test_record_exchange_torch_rccl_group(tmp_path):
    """The fallback bench.py takes when the library's RCCL communicator cannot start: the same overlapped,
    double-buffered exchange through a torch.distributed "nccl" (RCCL) process group, device to device.
    World 1 in a fresh process (one GPU here); three steps of gjkepa_batch_device, each step's gathered
    records equal to that step's."""
    import subprocess
    import sys
    pkg = os.path.join(ROOT, "collision-detect-gjk-epa_amd")
    f = tmp_path / "rccl_group.py"
    f.write_text(_TORCH_RCCL_SCRIPT)
    p = subprocess.run([sys.executable, str(f), pkg, "29557"], capture_output=True, text=True, timeout=110,
                       env=dict(os.environ, MASTER_ADDR="127.0.0.1"))
    assert p.returncode == 0 and p.stdout.strip().endswith("ok"), (p.stdout[-2000:], p.stderr[-3000:])


def test_two_rank_bench_verifies_its_exchange(tmp_path):
    """bench.py at N = 2 (torch.distributed.run, one process per rank, gloo control plane, both ranks
    on this box's one GPU, host-staged record exchange): each rank runs its shard through the library
    on the GPU; the line it prints carries the exchange's own check (every rank holds every other
    rank's records, rank 0's gathered buffer matches the oracle on a subsample of each shard) and the
    per-rank kernel / gather times."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29541", os.path.join(root, "bench.py"),
           "--gpus", "2", "--backend", "gloo", "--steps", "2", "--warmup", "1", "--pairs-per-gpu", "65536",
           "--cpu-sample", "2048"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env, cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-3000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("{")][-1]
    r = json.loads(line)
    assert r["n_gpus"] == 2 and r["config"]["total_pairs"] == 2 * 65536
    ps = r["parity_sample"]
    assert ps["gather_consistent"] and ps["all_equal"] and ps["bitexact_records"] == 1.0, ps
    assert ps["pairs"] == 2 * 2048
    assert sorted(x["rank"] for x in r["per_rank"]) == [0, 1]
    assert all(x["kernel_ms"] > 0 and x["gather_ms"] > 0 for x in r["per_rank"])


@pytest.mark.timeout(420)
def test_c3_whole_job_eight_ranks(tmp_path):
    """bench.py --gpus 8 (C3: 2^21 pairs per rank, 2^24 in all) under torch.distributed.run: eight
    processes on this box's one GPU, host-staged all-gather (gloo).  The line checks its own exchange:
    every rank's hash of every slot agrees, and rank 0's gathered buffer matches the oracle on the first
    2048 pairs of every shard."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    log = os.path.join(ROOT, "gpurun_out", "c3_bench.log") if os.path.isdir(os.path.join(ROOT, "gpurun_out")) \
        else str(tmp_path / "c3_bench.log")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(C3_RANKS),
           "--master-addr", "127.0.0.1", "--master-port", "29553", os.path.join(ROOT, "bench.py"),
           "--gpus", str(C3_RANKS), "--backend", "gloo", "--steps", "1", "--warmup", "0", "--cpu-sample", "2048"]
    _log("C3: 8-rank bench starting")
    with open(log, "w") as lf:
        p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=lf, text=True, timeout=400, env=env, cwd=str(tmp_path))
    assert p.returncode == 0, open(log).read()[-3000:]
    r = json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][-1])
    _log(f"C3: bench done, {r['value']} M queries/s over {r['n_gpus']} ranks")
    assert r["n_gpus"] == C3_RANKS and r["config"]["total_pairs"] == C3_RANKS * PER_RANK
    assert r["config"]["pairs_per_gpu"] == PER_RANK and r["config"]["workload"].startswith("C3")
    ps = r["parity_sample"]
    assert ps["gather_consistent"] and ps["all_equal"] and ps["bitexact_records"] == 1.0, ps
    assert ps["shards"] == C3_RANKS and ps["pairs"] == C3_RANKS * 2048
    assert sorted(x["rank"] for x in r["per_rank"]) == list(range(C3_RANKS))
    _c3["slot_sha16"] = {x["rank"]: x["slot_sha16"] for x in r["per_rank"]}


@pytest.mark.timeout(420)
def test_c3_gathered_job_equals_contiguous_run(orc):
    """The 2^24-pair C3 job in this process: one contiguous gjkepa_batch, and gjkepa_batch_multi over
    eight shards of device 0 (the one-process multi-device entry), byte-identical to each other; each
    shard's records hash to the slot the 8-rank bench gathered for that rank; the oracle agrees on 1024
    pairs spread over every shard."""
    if "slot_sha16" not in _c3:
        pytest.skip("needs test_c3_whole_job_eight_ranks")
    total = C3_RANKS * PER_RANK
    _log("C3: generating 2^24 pairs")
    whole = gjkepa.synth_pairs(SEED, total, 32, 32, 2.5)
    _log("C3: contiguous gjkepa_batch")
    ref = gjkepa.gjkepa_batch(whole, 2, 1.0)
    _log("C3: gjkepa_batch_multi over 8 shards of device 0")
    multi = gjkepa.gjkepa_batch_multi(whole, [0] * C3_RANKS, 2, 1.0)
    assert multi.tobytes() == ref.tobytes()
    del multi
    raw = ref.view(np.uint8).reshape(-1)
    slot = PER_RANK * ref.itemsize
    for s in range(C3_RANKS):
        first, count = gjkepa.shard_range(total, C3_RANKS, s)
        assert (first, count) == (s * PER_RANK, PER_RANK)
        h = hashlib.sha256(raw[s * slot:(s + 1) * slot].tobytes()).hexdigest()[:16]
        assert h == _c3["slot_sha16"][s], s
        sub = first + np.arange(0, count, count // 1024)[:1024]
        o = orc.gjkepa_batch(gjkepa.HullPool(whole.verts, whole.hull_off, whole.hull_cnt, whole.pairs[sub]), 2, 1.0)
        assert ref[sub].tobytes() == o.tobytes(), s
    _log("C3: contiguous run, 8-shard run and 8-rank gather identical")
