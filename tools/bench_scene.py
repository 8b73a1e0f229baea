#!/usr/bin/env python3
"""Benchmark of the device broad phase and of a whole collision step built
on it, one MI355X.

Scene S1 (gjkepa_synth_scene, seed 0x6A4B5C1D): 2^20 hulls x 32 unit-sphere vertices, centres
uniform in a cube sized for ~4 candidate pairs per hull (box = (N*113/6)^(1/3)).
  broadphase  step = gjkepa_broadphase_device over the scene (hulls resident in HBM)
  collide     step = broad phase, read the pair count, narrow phase (gjkepa_batch_device) on the
              device-resident list: the reference caller's all-pairs GJKEPA loop, on the GPU
Prints one JSON line per leg (bench.py's format); value = M hulls/s per step; the narrow leg also
reports M pair queries/s.  cpu_baseline: the oracle broad phase (+ narrow phase on a sample).

    python tools/bench_scene.py [--hulls N] [--steps K]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "collision-detect-gjk-epa_amd"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402

import gjkepa  # noqa: E402

SEED = 0x6A4B5C1D
PEAK_HBM_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hulls", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    import torch

    n = args.hulls
    box = (n * 113 / 6) ** (1 / 3)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    gjkepa.load()
    pool = gjkepa.synth_scene(SEED, n, 32, 32, box)
    v = torch.from_numpy(pool.verts).to(dev)
    off = torch.from_numpy(pool.hull_off).to(dev)
    cnt = torch.from_numpy(pool.hull_cnt).to(dev)
    cap = 8 * n
    pairs = torch.empty((cap, 2), dtype=torch.int32, device=dev)
    npair = torch.zeros(1, dtype=torch.int64, device=dev)
    wsb = gjkepa.broadphase_workspace_bytes(n, cap)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream

    def broad():
        gjkepa.broadphase_device(gjkepa.DTYPE_F32, v.data_ptr(), off.data_ptr(), cnt.data_ptr(), n, pairs.data_ptr(),
                                 cap, npair.data_ptr(), ws.data_ptr(), wsb, sp)

    broad()
    torch.cuda.synchronize(dev)
    npairs = int(npair.item())
    out = torch.empty(npairs * 128, dtype=torch.uint8, device=dev)
    nws = gjkepa.workspace_bytes(npairs)
    nw = torch.empty(nws, dtype=torch.uint8, device=dev)

    def narrow(m):
        gjkepa.gjkepa_batch_device(2, 1.0, gjkepa.DTYPE_F32, gjkepa.PREC_F64, v.data_ptr(), off.data_ptr(),
                                   cnt.data_ptr(), pairs.data_ptr(), m, out.data_ptr(), nw.data_ptr(), nws, sp)

    def timed(fn):
        for _ in range(args.warmup):
            fn()
        torch.cuda.synchronize(dev)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        t0 = time.perf_counter()
        for a, b in ev:
            a.record(stream)
            fn()
            b.record(stream)
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / args.steps, sum(a.elapsed_time(b) for a, b in ev) / args.steps

    def collide():
        broad()
        m = int(npair.item())          # the one host read of the step: the narrow phase's batch size
        narrow(m)

    wall_b, ms_b = timed(broad)
    wall_c, ms_c = timed(collide)
    recs = np.frombuffer(out.cpu().numpy().tobytes(), dtype=gjkepa.REC64)
    alg = 12.0 * pool.hull_cnt.astype(np.float64).sum() + n * 12 + 8.0 * npairs
    common = {"n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "higher_is_better": True, "scaling": "weak",
              "vs_baseline": None, "dtype": "f64", "data": "synthetic"}
    cfg = {"workload": f"S1: {n} hulls x 32 unit-sphere vertices, centres uniform in [0,{box:.1f})^3, fp32 storage",
           "hulls": n, "seed": SEED, "candidate_pairs": npairs}
    res_b = {"metric": "M hulls/sec through the device broad phase (SURVEY §8 f2)", "value": round(n / wall_b / 1e6, 3),
             "unit": "M hulls/s", "ms_per_step": round(1e3 * wall_b, 4), **common, "config": cfg,
             "roofline": {"bound": "hbm", "achieved": round(alg / (ms_b * 1e-3) / 1e9, 3), "peak": PEAK_HBM_GBS,
                          "unit": "GB/s", "frac": round(alg / (ms_b * 1e-3) / 1e9 / PEAK_HBM_GBS, 6), "traffic": None,
                          "bytes_per_hull": round(alg / n, 1), "kernel_ms": round(ms_b, 4),
                          "kernel": "sphere + radix sort + sweep (count, scan, emit) + pair sort (HIP events)"}}
    res_c = {"metric": "M hulls/sec through a whole collision step (broad + narrow phase)",
             "value": round(n / wall_c / 1e6, 3), "unit": "M hulls/s", "ms_per_step": round(1e3 * wall_c, 4), **common,
             "config": cfg, "pair_queries_per_s_M": round(npairs / wall_c / 1e6, 3), "device_ms": round(ms_c, 4),
             "hit_rate": round(float((recs["collision"] != 0).mean()), 4)}
    if not args.no_cpu:
        import oracle  # checker / CPU baseline only
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(os.cpu_count() or 1, 16)
        t = time.perf_counter()
        rp, rn = oracle.broadphase(pool.verts, pool.hull_off, pool.hull_cnt, nthreads=threads)
        ct = time.perf_counter() - t
        res_b["cpu_baseline"] = {"value": round(n / ct / 1e6, 4), "unit": "M hulls/s", "cores": threads, "kind": "port",
                                 "sample": f"the whole scene, oracle_broadphase (grid + exact test, OpenMP), {ct:.2f} s"}
        gp = pairs[:npairs].cpu().numpy()
        res_b["parity"] = {"pairs": npairs, "identical_list": bool(rn == npairs and np.array_equal(gp, rp))}
        m = min(npairs, 1 << 18)
        sub = gjkepa.HullPool(pool.verts, pool.hull_off, pool.hull_cnt, gp[:m])
        t = time.perf_counter()
        cref = oracle.gjkepa_batch(sub, 2, 1.0, threads)
        nt = time.perf_counter() - t
        per_pair = nt / m
        res_c["cpu_baseline"] = {"value": round(n / (ct + per_pair * npairs) / 1e6, 4), "unit": "M hulls/s",
                                 "cores": threads, "kind": "port",
                                 "sample": f"oracle broad phase on the whole scene ({ct:.2f} s) + oracle narrow phase "
                                           f"on the first {m} pairs ({nt:.2f} s), extrapolated to {npairs} pairs"}
        res_c["parity_sample"] = {"pairs": m, "bitexact": bool(recs[:m].tobytes() == cref.tobytes())}
    print(json.dumps(res_b), flush=True)
    print(json.dumps(res_c), flush=True)


if __name__ == "__main__":
    main()
