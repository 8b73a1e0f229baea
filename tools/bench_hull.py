#!/usr/bin/env python3
"""Benchmark of the batched convex-hull module, one MI355X.

A step is one gjkepa_hull_batch_device call over the whole cloud batch (points, offsets and the
output buffers resident in HBM).  Workloads (gjkepa_synth_clouds, seed 0x6A4B5C1D):
  H1: 2^20 clouds of 64 points uniform in the unit ball (kernel tier 0, mostly interior points)
  H2: 2^18 clouds of 256 points uniform in the ball (tier 1)
  H3: 2^16 clouds of 256 points on the unit sphere (tier 1, every point a hull vertex: worst case)
Prints one JSON line in bench.py's format: value = M hulls/s, roofline from HIP events on the
launch stream, cpu_baseline = the oracle restatement on the host cores over a bounded sample, and
a bit-exact parity check of the first clouds against the oracle.

    python tools/bench_hull.py [--config H1|H2|H3] [--steps K] [--warmup W]
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
CONFIGS = {   # n_clouds, n_min, n_max, shape, description
    "H1": (1 << 20, 64, 64, 0, "2^20 clouds x 64 points uniform in the unit ball"),
    "H2": (1 << 18, 256, 256, 0, "2^18 clouds x 256 points uniform in the unit ball"),
    "H3": (1 << 16, 256, 256, 1, "2^16 clouds x 256 points on the unit sphere (all extreme)"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=sorted(CONFIGS), default="H1")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--clouds", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    import torch

    n, lo, hi, shape, desc = CONFIGS[args.config]
    n = args.clouds or n
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    gjkepa.load()
    pool = gjkepa.synth_clouds(SEED, n, lo, hi, shape, dtype=np.float32)
    foff = gjkepa.hull_face_offsets(pool.cloud_cnt)
    nslots = int(foff[-1] + 2 * int(pool.cloud_cnt[-1]) - 4)
    p = torch.from_numpy(pool.verts).to(dev)
    off = torch.from_numpy(pool.cloud_off).to(dev)
    cnt = torch.from_numpy(pool.cloud_cnt).to(dev)
    fo = torch.from_numpy(foff).to(dev)
    faces = torch.empty((nslots, 3), dtype=torch.int32, device=dev)
    nf = torch.empty(n, dtype=torch.int32, device=dev)
    nv = torch.empty(n, dtype=torch.int32, device=dev)
    st = torch.empty(n, dtype=torch.int8, device=dev)
    hv = torch.empty_like(p)
    vi = torch.empty(pool.verts.size, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)

    def launch():
        gjkepa.hull_batch_device(gjkepa.DTYPE_F32, p.data_ptr(), off.data_ptr(), cnt.data_ptr(), n, fo.data_ptr(),
                                 faces.data_ptr(), nf.data_ptr(), nv.data_ptr(), st.data_ptr(), hv.data_ptr(),
                                 vi.data_ptr(), stream.cuda_stream)

    for _ in range(args.warmup):
        launch()
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for a, b in ev:
        a.record(stream)
        launch()
        b.record(stream)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    value = n * args.steps / elapsed / 1e6

    nfh, nvh, sth = nf.cpu().numpy(), nv.cpu().numpy(), st.cpu().numpy()
    # algorithmic bytes: points (fp32 SoA) + offset/count + face offset, written faces, counts/status,
    # hull pool entry (fp32) and vertex indices
    alg = (12.0 * pool.cloud_cnt.astype(np.float64).sum() + n * (8 + 4 + 8) + 12.0 * nfh.sum() + n * 9
           + 12.0 * nvh.sum() + 4.0 * nvh.sum())
    achieved = alg / (kern_ms * 1e-3) / 1e9
    result = {
        "metric": "M convex hulls/sec (batched QuickHull, SURVEY §8 f1)", "value": round(value, 4),
        "unit": "M hulls/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": f"{args.config}: {desc}, fp32 storage, fp64 compute", "clouds": n, "seed": SEED},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_HBM_GBS, 6), "traffic": None,
                     "bytes_per_hull": round(alg / n, 1), "kernel_ms": round(kern_ms, 4),
                     "kernel": "hull_kernel tiers 0 + 1 (HIP events on the launch stream)"},
        "hull_vertices_mean": round(float(nvh.mean()), 2), "faces_mean": round(float(nfh.mean()), 2),
        "status_counts": {int(k): int(v) for k, v in zip(*np.unique(sth, return_counts=True))},
    }
    if not args.no_cpu:
        import oracle  # checker / CPU baseline only
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(os.cpu_count() or 1, 16)
        m = min(n, 1 << 16)
        sub = slice(0, m)
        t = time.perf_counter()
        r = oracle.hull_batch(pool.verts, pool.cloud_off[sub], pool.cloud_cnt[sub], threads)
        ct = time.perf_counter() - t
        result["cpu_baseline"] = {"value": round(m / ct / 1e6, 4), "unit": "M hulls/s", "cores": threads, "kind": "port",
                                  "sample": f"first {m} clouds of the same batch, oracle_hull_batch (fp64, OpenMP over "
                                            f"clouds), {ct:.2f} s wall"}
        k = min(m, 4096)
        fg = faces.cpu().numpy()
        same = bool(np.array_equal(nfh[:k], r["n_faces"][:k]) and np.array_equal(nvh[:k], r["n_verts"][:k])
                    and np.array_equal(sth[:k], r["status"][:k]))
        for c in range(k):
            if not same:
                break
            a, b = int(foff[c]), int(foff[c]) + int(nfh[c])
            same = np.array_equal(fg[a:b], r["faces"][a:b])
        result["parity_sample"] = {"clouds": k, "bitexact": same}
    print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
