#!/usr/bin/env python3
"""Benchmark: M convex-pair GJK+EPA queries/s on N x MI355X (BASELINE.json metric).

Workload (N=1) = BASELINE config C2: 2^20 random 32-vertex convex-hull pairs, fp32 vertex storage,
version_=2, TOL_FF_=1.0, hull B centre offset r ~ U[0, 2.5] (seed 0x6A4B5C1D).
N>1 defaults to config C3: the same distribution, 2^21 pairs per GPU (2^24 on 8 GPUs).
A "step" is one pass of the hot path (gjkepa_batch_device: the tiered GJK/EPA kernels) over the
whole batch, with hulls, pair list and output already resident in HBM.  For N > 1 each rank owns
a contiguous shard of the config's pairs per GPU (weak scaling; the library's gjkepa_shard_range) and
every step's contact records are all-gathered over xGMI by the library's RCCL communicator
(gjkepa_comm_* / gjkepa_allgather_records_device: config C3's exchange).  The gather of step i runs
on its own stream while step i+1's kernels run (two record buffers, gathered in place); the timed
region ends after the last gather has completed, so every step's exchange is inside it.
torch.distributed (gloo) is the control plane only: RCCL id broadcast, barriers, max over ranks.
`--backend gloo` is the one-GPU rehearsal: ranks may share a device, records gathered via host.

The roofline is the dominant kernel's: the library's launch timing (gjkepa_launch_timing: HIP events
recorded around every kernel launch, on the stream that launch goes to) gives each launch's duration
inside the timed region; the kernel whose launches span the most time per step is dominant, and its
`achieved` = algorithmic bytes of the pairs one launch serves (route tally) / its mean launch duration.
The whole chain's figure is reported beside it (`roofline.chain`).

Extra legs (not timed in `value`), rank 0 at N=1: configs C4 and C5 on the same GPU (throughput, their
own dominant kernel, an oracle parity sample), fp32 compute, warm start, the host-buffer entry, and a
CPU baseline — the oracle restatement (kind "port") over a bounded sample of the same pairs, which also
re-checks GPU/CPU parity on that sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "collision-detect-gjk-epa_amd"))

import numpy as np  # noqa: E402

import gjkepa  # noqa: E402
import shard  # noqa: E402

SEED = 0x6A4B5C1D
PEAK_HBM_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "M convex-pair GJK+EPA queries/sec at 1/2/4/8 MI355X; % HBM roofline"


# BASELINE.json configs: (hull n_min, n_max, centre offset r_max, default pairs per GPU)
CONFIGS = {
    "C2": (32, 32, 2.5, 1 << 20, "1M random 32-vertex convex-hull pairs"),
    "C3": (32, 32, 2.5, 1 << 21, "C2 distribution, 2^21 32-vertex pairs per GPU (16M on 8 GPUs), "
                                 "contact records all-gathered over xGMI"),
    "C4": (8, 256, 2.5, 4 << 20, "4M pairs, mixed hull sizes 8-256 vertices"),
    "C5": (32, 128, 0.3, 1 << 20, "deep-overlap pairs (r~U[0,0.3]), 32-128-vertex hulls, EPA-heavy"),
}


def algorithmic_bytes_per_query(mean_verts_per_pair: float, vert_bytes: int, rec_bytes: int) -> float:
    """Bytes one query must move through HBM: both hulls' vertices (SoA), the pair's two hull
    indices, the two hulls' (offset, count) and the contact record it writes."""
    return vert_bytes * 3 * mean_verts_per_pair + 2 * 4 + 2 * (8 + 4) + rec_bytes


def moved_copy(pool, delta: float, seed: int) -> np.ndarray:
    """The pool's vertices with hull B of every pair translated by a random vector of length delta."""
    rng = np.random.default_rng(seed)
    v = pool.verts.astype(np.float64).copy()
    hb = pool.pairs[:, 1].astype(np.int64)
    d = rng.normal(size=(len(hb), 3))
    d *= delta / np.linalg.norm(d, axis=1, keepdims=True)
    cnt = pool.hull_cnt[hb].astype(np.int64)
    idx = np.repeat(pool.hull_off[hb], cnt) + (np.arange(cnt.sum()) - np.repeat(np.cumsum(cnt) - cnt, cnt))
    for j in range(3):
        v[idx + j * np.repeat(cnt, cnt)] += np.repeat(d[:, j], cnt)
    return v.astype(pool.verts.dtype)


WS_COUNTERS, WS_TALLY = gjkepa.WS_COUNTERS, gjkepa.WS_TALLY     # workspace header (uint32 words)
ROUTE_EPA0, ROUTE_CT0 = 0x10, 0x20


def served_pairs(r, tally: np.ndarray, recs, shares: dict) -> float:
    """Pairs one launch served: its route code's tally (workspace header, last chain), split across the
    parts of a parted tier by the share of the batch's hits inside each part's pair range."""
    k, code = r["kernel"].decode(), int(r["route_code"])
    if k == "gjk" and int(r["tier"]) == 0:
        return float(r["n_pairs"])
    if code < 0 or code >= len(tally):
        return 0.0
    tot = float(tally[code])
    key = (k, int(r["tier"]), code)
    if key in shares and shares[key] > 0:
        f, c = int(r["first_pair"]), int(r["n_pairs"])
        hits = recs["collision"][f:f + c] != 0
        return tot * float(hits.sum()) / shares[key]
    return tot


def busy_span(rs) -> float:
    """Time covered by the union of the launches' [start, end] intervals (concurrent launches once)."""
    iv = sorted((float(r["start_ms"]), float(r["end_ms"])) for r in rs)
    tot, cs, ce = 0.0, None, None
    for s, e in iv:
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + (ce - cs if ce is not None else 0.0)


def dominant_kernel(lt: np.ndarray, tally: np.ndarray, recs, bpq: float, pmc: dict | None) -> dict:
    """The kernel (kind, tier) with the most launch time per chain (sum of its launches' durations), from
    the launch timing of the measured steps (gjkepa_launch_timing_read records); its wall span is the
    union of its launches' intervals per chain (two concurrent parts count once)."""
    chains = sorted(set(int(c) for c in lt["chain"]))
    groups: dict = {}
    for r in lt:
        groups.setdefault((r["kernel"].decode(), int(r["tier"])), []).append(r)
    best, best_busy = None, -1.0
    for key, rs in groups.items():
        busy = sum(float(r["end_ms"]) - float(r["start_ms"]) for r in rs) / len(chains)
        if busy > best_busy:
            best, best_busy = key, busy
    rs = groups[best]
    best_span = float(np.mean([busy_span([r for r in rs if int(r["chain"]) == c]) for c in chains]))
    # parts of one route code in several pair ranges: hits per range apportion the code's tally
    by_code: dict = {}
    for r in rs:
        if int(r["chain"]) == chains[-1]:
            by_code.setdefault((best[0], best[1], int(r["route_code"])), []).append(r)
    shares = {}
    for key, lst in by_code.items():
        if len(lst) > 1:
            shares[key] = float(sum(int((recs["collision"][int(r["first_pair"]):int(r["first_pair"]) + int(r["n_pairs"])] != 0).sum())
                                    for r in lst))
    last = [r for lst in by_code.values() for r in lst]
    served = [served_pairs(r, tally, recs, shares) for r in last]
    durs = np.array([float(r["end_ms"]) - float(r["start_ms"]) for r in rs])
    per_chain = len(rs) / len(chains)
    pairs_per_launch = float(np.sum(served)) / max(len(last), 1)
    launch_ms = float(durs.mean())
    achieved = pairs_per_launch * bpq / (launch_ms * 1e-3) / 1e9
    span_achieved = float(np.sum(served)) * bpq / (best_span * 1e-3) / 1e9 if best_span > 0 else 0.0
    out = {"kernel": f"{best[0]} tier {best[1]}", "launches_per_step": per_chain,
           "pairs_per_launch": round(pairs_per_launch, 1), "pairs_per_step": float(np.sum(served)),
           "launch_ms": round(launch_ms, 4), "launch_ms_each": [round(float(d), 4) for d in durs[-len(last):]],
           "wall_span_ms": round(best_span, 4), "bytes_per_pair": round(bpq, 1),
           "achieved": round(achieved, 3), "frac": round(achieved / PEAK_HBM_GBS, 6),
           "span_achieved": round(span_achieved, 3), "span_frac": round(span_achieved / PEAK_HBM_GBS, 6),
           "method": "HIP events around each launch (gjkepa_launch_timing) over the timed steps; pairs = the "
                     "launch's route-code tally in the workspace (parts: split by the hits in each part's range); "
                     "achieved = pairs per launch x bytes per pair / mean launch duration; span_* = per step, "
                     "over the wall time its launches cover (the union of their intervals)"}
    # the same kernel in the committed PMC run (same library source hash): its traffic per launch and its
    # VALU-busy share priced against the wall span of its launches
    if pmc:
        want = {"epa": "epa_kernel", "gjk": "gjk_kernel", "contact": "contact_kernel", "redo": "redo_kernel"}.get(best[0], "?")
        cand = [(v.get("seconds", 0.0), k, v) for k, v in pmc.get("kernels", {}).items() if want in k]
        if cand:
            _, name, v = max(cand, key=lambda x: x[0])
            disp = v.get("dispatches_per_chain") or 1.0
            out["pmc"] = {"kernel": name, "traffic_per_launch": (2.0 * v.get("FETCH_SIZE", 0.0) + v.get("WRITE_SIZE", 0.0)) * 1024.0 / disp,
                          "valu_instr_per_pair": v.get("SQ_INSTS_VALU", 0.0) / max(float(np.sum(served)), 1.0),
                          "salu_per_valu": v.get("SQ_INSTS_SALU", 0.0) / max(v.get("SQ_INSTS_VALU", 1.0), 1.0),
                          "busy_frac_span": v.get("SQ_ACTIVE_INST_VALU", 0.0) * 4.0 / (1024 * best_span * 1e-3 * 2.4e9)
                          if best_span > 0 else None,
                          "note": "PMC counters of the largest-time instantiation of this kernel (profiles/pmc_traffic.json), "
                                  "summed over its dispatches per chain; busy_frac_span = SQ_ACTIVE_INST_VALU x 4 over "
                                  "1024 SIMDs x the live wall span x 2.4 GHz"}
    return out


def read_tally(ws) -> np.ndarray:
    return ws[4 * WS_COUNTERS:4 * (WS_COUNTERS + WS_TALLY)].cpu().numpy().view(np.uint32).copy()


def pmc_entry(precision: str, config: str, n: int, lib_src: str) -> dict | None:
    """The committed PMC summary of this (precision, config, batch) at the loaded library's source hash."""
    prof = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(prof):
        return None
    try:
        pj = json.load(open(prof)).get(f"{precision}_{config}_{n}")
    except (OSError, ValueError):
        return None
    return pj if pj and pj.get("src") == lib_src else None


def host_cpus() -> dict:
    """Host cores the CPU baseline may use: the process's affinity set, capped by a cgroup CPU quota
    (a GPU box exposes the whole machine in os.cpu_count() but grants a share of it), and the CPU model."""
    nproc = os.cpu_count() or 1
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    usable = min(aff, quota) if quota else aff
    if env:
        usable = min(usable, env)
    return {"usable": usable, "nproc": nproc, "affinity": aff, "cgroup": quota, "model": model,
            "omp_num_threads": env or None}


def verify_exchange(result, args, ex, comm, dist, world, rank, n, prec, rec_bytes, kern_ms_local, cfg, stream):
    """N > 1, after the timed region: the record exchange checks itself.

    - consistency: every rank hashes each rank's slot of its gathered buffer (last step); rank s's own
      slot holds what its kernels wrote (the gather runs in place), so every rank's hash of slot s must
      equal rank s's own hash of it;
    - parity: rank 0 re-runs a subsample of every shard through the oracle (fp64 compute) and compares
      it byte for byte with that shard's slot of its gathered buffer;
    - timing: per-rank kernel ms (HIP events on the launch stream, mean per step) and the time of one
      more stand-alone all-gather of the same buffer (events on the exchange stream; host clock for gloo).
    """
    import hashlib
    import time as _t

    import torch
    gath = ex.last_gathered.cpu().numpy()
    slot = n * rec_bytes
    mine = [hashlib.sha256(gath[s * slot:(s + 1) * slot].tobytes()).hexdigest()[:16] for s in range(world)]
    allh = [None] * world
    dist.all_gather_object(allh, mine)
    consistent = all(allh[r][s] == allh[s][s] for r in range(world) for s in range(world))
    # one more gather of the same buffer, timed
    b = ex.cur
    if ex.overlap:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(ex.stream)
        if comm is not None:
            comm.allgather_records(prec, ex.local[b].data_ptr(), ex.gathered[b].data_ptr(), ex.count, ex.stream.cuda_stream)
        else:
            with torch.cuda.stream(ex.stream):
                dist.all_gather_into_tensor(ex.gathered[b], ex.local[b], group=ex.device_group)
        e1.record(ex.stream)
        e1.synchronize()
        gather_ms = e0.elapsed_time(e1)
    else:
        t = _t.perf_counter()
        g = torch.empty(ex.gathered[b].numel(), dtype=torch.uint8)
        dist.all_gather_into_tensor(g, ex.local[b].cpu(), group=ex.group)
        ex.gathered[b].copy_(g)
        torch.cuda.synchronize()
        gather_ms = 1e3 * (_t.perf_counter() - t)
    per = [None] * world
    dist.all_gather_object(per, {"rank": rank, "kernel_ms": round(kern_ms_local, 4), "gather_ms": round(gather_ms, 4),
                                 "slot_sha16": mine[rank]})
    ps = {"gather_consistent": bool(consistent), "shards": world}
    if rank == 0 and prec == gjkepa.PREC_F64 and not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle  # checker only
        nmin, nmax, rmax = cfg
        m = min(n, args.cpu_sample or 8192)
        threads = host_cpus()["usable"]
        eq_total, bad = 0, 0
        for s in range(world):
            first_s, _ = shard.shard_range(n * world, world, s)
            sub = gjkepa.synth_pairs(SEED, m, nmin, nmax, rmax, first_pair=first_s, dtype=np.float32)
            ref = np.frombuffer(oracle.gjkepa_batch(sub, args.version, 1.0, threads).tobytes(), np.uint8).reshape(m, -1)
            got = gath[s * slot:s * slot + m * rec_bytes].reshape(m, -1)
            eqr = (got == ref).all(axis=1)
            eq_total += int(eqr.sum())
            bad += int((~eqr).sum())
        ps.update({"pairs": m * world, "pairs_per_shard": m, "bitexact_records": eq_total / (m * world),
                   "all_equal": bad == 0 and consistent, "against": "oracle, every shard's slot of rank 0's gathered buffer"})
    result["parity_sample"] = ps
    result["per_rank"] = per


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", choices=sorted(CONFIGS), default=None,
                    help="default: C2 on one GPU, C3 (2^21 pairs per GPU + all-gather) when --gpus > 1")
    ap.add_argument("--pairs-per-gpu", type=int, default=0, help="0: the config's size")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="N>1 record exchange: nccl = the library's RCCL all-gather, gloo = host-staged rehearsal")
    ap.add_argument("--version", type=int, default=2)
    ap.add_argument("--precision", choices=["f64", "f32"], default="f64")
    ap.add_argument("--no-gather", action="store_true", help="skip the RCCL all-gather for N>1")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-f32-leg", action="store_true", help="skip the fp32-compute side measurement")
    ap.add_argument("--no-warm-leg", action="store_true", help="skip the warm-start side measurement")
    ap.add_argument("--cpu-sample", type=int, default=0, help="pairs for the CPU baseline (0: the whole batch)")
    ap.add_argument("--legs", default="C4,C5", help="N=1: extra configs run on the same GPU after the main one "
                                                   "(comma list; 'none' to skip)")
    ap.add_argument("--leg-sample", type=int, default=65536, help="pairs of each leg checked against the oracle")
    ap.add_argument("--launch-timing", choices=["timed", "separate", "off"], default="separate",
                    help="separate (default): the launch events in a second pass of the same steps right after the "
                         "timed ones (they cost ~0.9%% on C2 when inside: profiles/r05/ab_launch_timing.txt); "
                         "timed: inside the timed steps")
    return ap.parse_args()


def run_leg(cfg: str, args, dev, stream, prec: int, lib_src: str) -> dict:
    """One more config on this GPU (N=1): its own batch resident in HBM, warmup, `steps` timed chains
    with launch timing, the dominant kernel, and an oracle parity sample of its first pairs."""
    import torch
    nmin, nmax, rmax, n, desc = CONFIGS[cfg]
    rec_bytes = gjkepa.load().gjkepa_record_bytes(prec)
    pool = gjkepa.synth_pairs(SEED, n, nmin, nmax, rmax, dtype=np.float32)
    verts = torch.from_numpy(pool.verts).to(dev)
    off = torch.from_numpy(pool.hull_off).to(dev)
    cnt = torch.from_numpy(pool.hull_cnt).to(dev)
    prs = torch.from_numpy(pool.pairs.reshape(-1)).to(dev)
    out = torch.zeros(n * rec_bytes, dtype=torch.uint8, device=dev)
    ws_bytes = gjkepa.workspace_bytes_for(n, gjkepa.large_pairs(pool))
    ws = torch.zeros(ws_bytes, dtype=torch.uint8, device=dev)
    sptr = stream.cuda_stream

    def launch():
        gjkepa.gjkepa_batch_device(args.version, 1.0, gjkepa.DTYPE_F32, prec, verts.data_ptr(), off.data_ptr(),
                                   cnt.data_ptr(), prs.data_ptr(), n, out.data_ptr(), ws.data_ptr(), ws_bytes, sptr)
    for _ in range(max(args.warmup, 1)):
        launch()
    torch.cuda.synchronize(dev)
    steps = max(1, min(args.steps, 10))
    inside = args.launch_timing == "timed"
    gjkepa.launch_timing(inside)
    t0 = time.perf_counter()
    for _ in range(steps):
        launch()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    if not inside:                                  # the same steps once more, with the launch events
        gjkepa.launch_timing(True)
        for _ in range(steps):
            launch()
        torch.cuda.synchronize(dev)
    gjkepa.launch_timing(False)
    lt = gjkepa.launch_timing_read()
    recs = np.frombuffer(out.cpu().numpy().tobytes(), dtype=gjkepa.record_dtype(prec))
    bpq = algorithmic_bytes_per_query(float(pool.hull_cnt.sum()) / n, 4, rec_bytes)
    chain_ms = float(np.mean([lt["end_ms"][lt["chain"] == c].max() for c in set(lt["chain"].tolist())]))
    r = {"config": cfg, "workload": f"{cfg}: {desc}", "pairs": n, "steps": steps,
         "value": round(n * steps / el / 1e6, 3), "unit": "M queries/s", "ms_per_step": round(1e3 * el / steps, 4),
         "chain_ms": round(chain_ms, 4), "bytes_per_query": round(bpq, 1),
         "hit_rate": round(float((recs["collision"] != 0).mean()), 4),
         "status_counts": {int(k): int(v) for k, v in zip(*np.unique(recs["status"], return_counts=True))},
         "dominant_kernel": dominant_kernel(lt, read_tally(ws), recs, bpq, pmc_entry(args.precision, cfg, n, lib_src))}
    pmc = pmc_entry(args.precision, cfg, n, lib_src)
    dom = r["dominant_kernel"]
    # the leg's own roofline block, as the main line's: the dominant kernel's achieved bytes against
    # the HBM peak, its PMC traffic per launch, and the chain's traffic / VALU issue from the same run
    r["roofline"] = {"bound": "hbm", "achieved": dom["achieved"], "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": dom["frac"], "traffic": dom.get("pmc", {}).get("traffic_per_launch"),
                     "kernel": dom["kernel"], "pmc_src": pmc["src"] if pmc else None}
    r["traffic_per_chain"] = pmc["bytes_per_launch"] if pmc else None
    r["valu_issue"] = ({"instr_per_query": round(pmc["valu_instr_per_query"], 1),
                        "issue_frac_pmc": round(pmc["valu_issue_frac"], 4),
                        "busy_frac_pmc": round(pmc["valu_busy_frac"], 4) if pmc.get("valu_busy_frac") else None}
                       if pmc else None)
    if prec == gjkepa.PREC_F64 and args.leg_sample > 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle  # checker only, after the timed steps
        m = min(n, args.leg_sample)
        sub = gjkepa.HullPool(pool.verts, pool.hull_off, pool.hull_cnt, pool.pairs[:m])
        ref = oracle.gjkepa_batch(sub, args.version, 1.0, host_cpus()["usable"])
        eq = np.frombuffer(recs[:m].tobytes(), np.uint8).reshape(m, -1) == np.frombuffer(ref.tobytes(), np.uint8).reshape(m, -1)
        r["parity_sample"] = {"pairs": m, "bitexact_records": float(eq.all(axis=1).mean()),
                              "all_equal": bool(eq.all()), "against": "oracle, the leg's first pairs"}
    del verts, off, cnt, prs, out, ws
    torch.cuda.empty_cache()
    return r


def main():
    args = parse()
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        print(f"warning: WORLD_SIZE={world} but --gpus={args.gpus}", file=sys.stderr)
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")          # control plane; the data path is the library's RCCL
        torch.cuda.set_device(local % max(torch.cuda.device_count(), 1))   # gloo rehearsal: ranks may share a GPU
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", torch.cuda.current_device())
    lib = gjkepa.load()

    if args.config is None:
        args.config = "C3" if max(world, args.gpus) > 1 else "C2"
    nmin, nmax, rmax, n_default, desc = CONFIGS[args.config]
    n = args.pairs_per_gpu or n_default
    prec = gjkepa.PREC_F64 if args.precision == "f64" else gjkepa.PREC_F32
    rec_bytes = lib.gjkepa_record_bytes(prec)
    first, _ = shard.shard_range(n * world, world, rank)      # gjkepa_shard_range
    pool = gjkepa.synth_pairs(SEED, n, nmin, nmax, rmax, first_pair=first, dtype=np.float32)
    verts = torch.from_numpy(pool.verts).to(dev)
    off = torch.from_numpy(pool.hull_off).to(dev)
    cnt = torch.from_numpy(pool.hull_cnt).to(dev)
    prs = torch.from_numpy(pool.pairs.reshape(-1)).to(dev)
    out = torch.zeros(n * rec_bytes, dtype=torch.uint8, device=dev)
    ws_bytes = gjkepa.workspace_bytes_for(n, gjkepa.large_pairs(pool))     # park slots only where pairs can park
    ws = torch.zeros(ws_bytes, dtype=torch.uint8, device=dev)
    # N > 1: every step's records are all-gathered (shard.RecordExchange); with the library's RCCL
    # communicator step i's gather overlaps step i+1's kernels (two record buffers), on gloo it is
    # staged through host memory
    ex, comm, dgroup, exchange = None, None, None, None
    if world > 1 and not args.no_gather:
        if args.backend == "nccl":
            # the library's RCCL communicator; if any rank cannot bring it up, every rank falls back to a
            # torch.distributed "nccl" (RCCL) group for the same device-to-device gather, and the line says so
            err = ""
            try:
                comm = shard.make_comm(world, rank, dev.index)
            except Exception as e:          # noqa: BLE001  (reported in the line, not hidden)
                err = f"{type(e).__name__}: {e}"
            ok = torch.tensor([0 if err else 1], dtype=torch.int32)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if int(ok[0]) == 1:
                exchange = "library RCCL communicator (gjkepa_allgather_records_device)"
            else:
                if comm is not None:
                    comm.close()
                    comm = None
                dgroup = dist.new_group(backend="nccl")
                errs = [None] * world
                dist.all_gather_object(errs, err)
                exchange = ("torch.distributed nccl (RCCL) group; the library communicator failed: " +
                            "; ".join(f"rank {r}: {e}" for r, e in enumerate(errs) if e))
        else:
            exchange = "gloo, host-staged (one-GPU rehearsal)"
        ex = shard.RecordExchange(n * rec_bytes, world, rank, dev, prec, comm=comm, device_group=dgroup)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream

    def launch(p, o):
        gjkepa.gjkepa_batch_device(args.version, 1.0, gjkepa.DTYPE_F32, p, verts.data_ptr(), off.data_ptr(),
                                   cnt.data_ptr(), prs.data_ptr(), n, o.data_ptr(), ws.data_ptr(), ws_bytes, sptr)

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]

    def step(i=None):
        o = ex.buffer(stream) if ex else out   # a reused buffer first waits for the gather that read it
        if i is not None:
            ev[i][0].record(stream)
        launch(prec, o)
        if i is not None:
            ev[i][1].record(stream)
        if ex:
            ex.submit(stream)

    def drain():
        if ex:
            ex.drain()

    for _ in range(args.warmup):
        step()
    drain()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    if args.launch_timing == "timed":
        gjkepa.launch_timing(True)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    drain()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    timing_ms_per_step = None
    if args.launch_timing == "separate":           # the same steps once more, with the launch events
        gjkepa.launch_timing(True)
        t1 = time.perf_counter()
        for i in range(args.steps):
            step()
        drain()
        torch.cuda.synchronize(dev)
        timing_ms_per_step = 1e3 * (time.perf_counter() - t1) / args.steps
    gjkepa.launch_timing(False)
    lt = gjkepa.launch_timing_read() if args.launch_timing != "off" else None
    tally = read_tally(ws)
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / max(args.steps, 1)
    kern_ms_local = kern_ms
    if dist:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
    ms_per_step = 1e3 * elapsed / args.steps
    total_pairs = n * world
    value = total_pairs * args.steps / elapsed / 1e6

    # statistics of the last step's records (rank-local)
    recs = np.frombuffer((ex.last if ex else out).cpu().numpy().tobytes(), dtype=gjkepa.record_dtype(prec))
    hit_rate = float((recs["collision"] != 0).mean())
    status_counts = {int(k): int(v) for k, v in zip(*np.unique(recs["status"], return_counts=True))}
    epa_iters = (recs["diag"] >> 8) & 0xFF
    epa_mean = float(epa_iters[recs["collision"] != 0].mean()) if hit_rate > 0 else 0.0

    bpq = algorithmic_bytes_per_query(float(pool.hull_cnt.sum()) / n, 4, rec_bytes)
    achieved = n * bpq / (kern_ms * 1e-3) / 1e9
    # HBM traffic and VALU issue of the same chain from the committed PMC run (tools/gpu_session.sh pmc +
    # tools/pmc_report.py), keyed by precision/config/batch size and stamped with the library's
    # source hash; null unless that hash is the one this process loaded (no figures from another build)
    traffic, valu, pmc_src = None, None, None
    lib_src = gjkepa.source_hash()
    pj = pmc_entry(args.precision, args.config, n, lib_src)
    if pj:
        pmc_src = pj["src"]
        traffic = pj["bytes_per_launch"]
        if pj.get("valu_instr"):
            valu = {"instr_per_query": round(pj["valu_instr_per_query"], 1),
                    "issue_frac_pmc": round(pj["valu_issue_frac"], 4),
                    "issue_frac_live": round(pj["valu_instr"] * 2.0 / (1024 * kern_ms * 1e-3 * 2.4e9), 4),
                    "busy_frac_pmc": round(pj["valu_busy_frac"], 4) if pj.get("valu_busy_frac") else None,
                    "traffic_raw_fetch": pj.get("fetch_bytes_raw"),
                    "note": "issue_frac: SQ_INSTS_VALU at the 2-cycle wave64 slot vs 1024 SIMDs x kernel time x "
                            "2.4 GHz (fp64 ops take 4: a lower bound); busy_frac: SQ_ACTIVE_INST_VALU (quad-cycles "
                            "x 4) over the summed kernel time (concurrent kernels overlap: see dominant_kernel.pmc "
                            "for the share over a wall span)"}
    chain = {"achieved": round(achieved, 3), "frac": round(achieved / PEAK_HBM_GBS, 6), "traffic": traffic,
             "valu_issue": valu, "bytes_per_query": round(bpq, 1), "queries_per_launch": n, "kernel_ms": round(kern_ms, 4),
             "kernel": "gjk + epa + contact kernel tiers (one launch chain; HIP events on the launch stream)",
             "pmc_src": pmc_src}
    dom = dominant_kernel(lt, tally, recs, bpq, pj) if lt is not None and len(lt) else None
    if dom is not None:
        dom["timing"] = args.launch_timing + ("" if timing_ms_per_step is None else f" (that pass: {timing_ms_per_step:.4f} ms/step)")
        # the dominant kernel's PMC traffic per launch (same source hash), or null
        roofline = {"bound": "hbm", "achieved": dom["achieved"], "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": dom["frac"], "traffic": dom.get("pmc", {}).get("traffic_per_launch"),
                    "kernel": dom["kernel"], "pmc_src": pmc_src, "chain": chain}
    else:
        roofline = {"bound": "hbm", **{k: chain[k] for k in ("achieved", "frac", "traffic", "kernel", "pmc_src")},
                    "peak": PEAK_HBM_GBS, "unit": "GB/s", "chain": chain}

    result = {
        "metric": METRIC, "value": round(value, 3), "unit": "M queries/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": args.precision, "data": "synthetic",
        "config": {"workload": f"{args.config}: {desc}, fp32 vertex storage, {args.precision} compute, "
                               f"version_={args.version}, TOL_FF_=1.0, hull B offset r~U[0,{rmax}]",
                   "hull_vertices": [nmin, nmax],
                   "pairs_per_gpu": n, "total_pairs": total_pairs, "seed": SEED,
                   "parallelism": f"shard{world}" + ("" if ex is None else "+rccl_allgather_overlapped" if ex.overlap
                                                       else "+gloo_allgather_host_staged"),
                   "vert_storage": "f32", "record_bytes": rec_bytes,
                   **({"exchange": exchange} if exchange else {})},
        "roofline": roofline,
        "dominant_kernel": dom,
        "hit_rate": round(hit_rate, 4), "epa_iters_mean": round(epa_mean, 2), "status_counts": status_counts,
        "lib": gjkepa.version_string(),
    }

    # fp32-compute side measurement (same batch), reported, never `value`
    if rank == 0 and world == 1 and not args.no_f32_leg and prec == gjkepa.PREC_F64:
        out32 = torch.zeros(n * 64, dtype=torch.uint8, device=dev)
        def l32():
            gjkepa.gjkepa_batch_device(args.version, 1.0, gjkepa.DTYPE_F32, gjkepa.PREC_F32, verts.data_ptr(),
                                       off.data_ptr(), cnt.data_ptr(), prs.data_ptr(), n, out32.data_ptr(),
                                       ws.data_ptr(), ws_bytes, sptr)
        l32()
        torch.cuda.synchronize(dev)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(stream)
        for _ in range(args.steps):
            l32()
        e.record(stream)
        torch.cuda.synchronize(dev)
        ms32 = s.elapsed_time(e) / args.steps
        redo = int(read_tally(ws)[0x2E])           # GJKEPA_ROUTE_REDO: pairs recomputed in fp64 by the last launch
        r32 = np.frombuffer(out32.cpu().numpy().tobytes(), dtype=gjkepa.REC32)
        # errors against the fp64 records of the same batch (byte-identical to the oracle: parity_sample),
        # with the full-batch gate of tests/test_gpu_parity.py::test_fp32_tolerance_sweep (tools/fp32_metrics.py)
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from fp32_metrics import fp32_report, passes
        rep = fp32_report(pool, r32, recs)
        v32 = n / (ms32 * 1e-3) / 1e6
        result["fp32_compute"] = {"value": round(v32, 3), "unit": "M queries/s", "over_fp64": round(v32 / value, 4),
                                  "redo_pairs": redo, "redo_frac": round(redo / n, 4), **rep, "gate_passed": passes(rep),
                                  "note": "opt-in (GJKEPA_PREC_F32; fp64 is the default precision): fp32 answers are kept only "
                                          "when certified to 1e-6 relative depth, the rest are recomputed in fp64 "
                                          "(redo_pairs; DESIGN.md section 6)"}

    # warm start: frames alternate between the batch and a copy with every hull B moved
    # by 1e-3; each frame's warm slots seed the next.  Cold = the same frames through batch_device.
    if rank == 0 and world == 1 and not args.no_warm_leg and prec == gjkepa.PREC_F64:
        moved = moved_copy(pool, 1e-3, SEED)
        frames = [verts, torch.from_numpy(moved).to(dev)]
        warm = torch.full((4 * n,), -1, dtype=torch.int32, device=dev)

        def frame(i, use_warm):
            args_ = (args.version, 1.0, gjkepa.DTYPE_F32, prec, frames[i % 2].data_ptr(), off.data_ptr(),
                     cnt.data_ptr(), prs.data_ptr(), n, out.data_ptr(), ws.data_ptr(), ws_bytes)
            if use_warm:
                gjkepa.gjkepa_batch_warm_device(*args_, warm.data_ptr(), sptr)
            else:
                gjkepa.gjkepa_batch_device(*args_, sptr)
        rates = {}
        for use_warm in (False, True):
            frame(0, use_warm)
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            for i in range(1, args.steps + 1):
                frame(i, use_warm)
            torch.cuda.synchronize(dev)
            rates[use_warm] = n * args.steps / (time.perf_counter() - t) / 1e6
        wr = np.frombuffer(out.cpu().numpy().tobytes(), dtype=gjkepa.REC64)
        hits = (wr["collision"] != 0) & (wr["status"] == 0)
        result["warm_start"] = {"value": round(rates[True], 3), "cold_value": round(rates[False], 3),
                                "unit": "M queries/s", "warm_started_hits": round(float(((wr["diag"] & 0xFF) == 0)[hits].mean()), 4),
                                "note": "frames alternate between the batch and hull B moved by 1e-3; "
                                        "gjkepa_batch_warm_device vs gjkepa_batch_device on the same frames"}

    # host-buffer entry point (gjkepa_batch: H2D copy of hulls/pairs, kernels, D2H of records):
    # the PCIe-inclusive rate, reported beside `value`, never as it
    if rank == 0 and world == 1 and not args.no_f32_leg:
        gjkepa.gjkepa_batch(pool, args.version, 1.0, precision=prec)
        t = time.perf_counter()
        for _ in range(2):
            gjkepa.gjkepa_batch(pool, args.version, 1.0, precision=prec)
        result["host_api"] = {"value": round(2 * n / (time.perf_counter() - t) / 1e6, 3), "unit": "M queries/s",
                              "note": "gjkepa_batch on host buffers, PCIe transfers included"}

    if dist and ex is not None:
        verify_exchange(result, args, ex, comm, dist, world, rank, n, prec, rec_bytes, kern_ms_local,
                        (nmin, nmax, rmax), stream)

    if rank == 0 and world == 1 and not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle  # checker / CPU baseline only
        m = min(args.cpu_sample, n) if args.cpu_sample > 0 else n
        sub = gjkepa.HullPool(pool.verts, pool.hull_off, pool.hull_cnt, pool.pairs[:m])
        host = host_cpus()
        threads = host["usable"]
        oracle.gjkepa_batch(gjkepa.HullPool(pool.verts, pool.hull_off, pool.hull_cnt, pool.pairs[:256]),
                            args.version, 1.0, threads)
        t = time.perf_counter()
        cref = oracle.gjkepa_batch(sub, args.version, 1.0, threads)
        ct = time.perf_counter() - t
        result["cpu_baseline"] = {
            "value": round(m / ct / 1e6, 4), "unit": "M queries/s", "cores": threads, "kind": "port",
            "sample": f"first {m} pairs of the same {args.config} batch, fp64 oracle restatement (oracle/gjkepa_oracle.c), "
                      f"OpenMP dynamic over pairs, {ct:.2f} s wall",
            "cpu_model": host["model"], "nproc": host["nproc"], "affinity": host["affinity"],
            "cgroup_cpus": host["cgroup"],
        }
        # one core, for a per-core figure (a bounded sample: ~1/64 of the pairs the threaded leg ran)
        m1 = max(256, m // max(threads, 1) // 4)
        t = time.perf_counter()
        oracle.gjkepa_batch(gjkepa.HullPool(pool.verts, pool.hull_off, pool.hull_cnt, pool.pairs[:m1]), args.version, 1.0, 1)
        result["cpu_baseline"]["per_core"] = {"value": round(m1 / (time.perf_counter() - t) / 1e6, 5), "pairs": m1}
        # the port against the reference itself (SURVEY §6 probe figures, GJK-only set, same container):
        # tools/cpu_calib.py -> profiles/r03/cpu_calib.json
        cal = os.path.join(ROOT, "profiles", "r03", "cpu_calib.json")
        if os.path.exists(cal):
            cj = json.load(open(cal))
            result["cpu_baseline"]["calibration"] = {
                "port_over_reference_1core": cj["port_over_reference_1core"],
                "port_over_reference_8core": cj["port_over_reference_8core"],
                "set": cj["set"], "source": "profiles/r03/cpu_calib.json (tools/cpu_calib.py)",
                "note": "the reference's GJK-only speed from SURVEY.md §6 (0.067 / 0.45 M pairs/s on 1 / 8 "
                        "container cores); the port is that many times faster per core on the same set"}
        if prec == gjkepa.PREC_F64:
            g = recs[:m]
            same = (g.tobytes() == cref.tobytes())
            eq = np.frombuffer(g.tobytes(), np.uint8).reshape(m, -1) == np.frombuffer(cref.tobytes(), np.uint8).reshape(m, -1)
            result["parity_sample"] = {"pairs": m, "bitexact_records": float(eq.all(axis=1).mean()), "all_equal": bool(same)}

    # configs C4 / C5 on the same GPU, after everything above (N=1 only)
    if rank == 0 and world == 1 and args.legs.lower() != "none":
        result["legs"] = {}
        for cfg in [c.strip() for c in args.legs.split(",") if c.strip()]:
            if cfg in CONFIGS and cfg != args.config:
                result["legs"][cfg] = run_leg(cfg, args, dev, stream, prec, lib_src)

    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.barrier()
        if comm is not None:
            comm.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
