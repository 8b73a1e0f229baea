#!/usr/bin/env python3
"""GPU box: what the resident query service costs a concurrent batch.

Times gjkepa_batch_device on the C2 batch (inputs in HBM, its own stream) alone, then while T threads
keep the service busy with single-pair gjkepa_query calls, then alone again after
gjkepa_query_service_stop; prints one JSON line.  usage: python tools/svc_concurrent.py [threads...]
"""
from __future__ import annotations

import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "collision-detect-gjk-epa_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import gjkepa  # noqa: E402
from bench import SEED  # noqa: E402


def main():
    threads = [int(a) for a in sys.argv[1:]] or [4, 16]
    n = 1 << 20
    dev = torch.device("cuda", 0)
    pool = gjkepa.synth_pairs(SEED, n, 32, 32, 2.5)
    v = torch.from_numpy(pool.verts).to(dev)
    o = torch.from_numpy(pool.hull_off).to(dev)
    c = torch.from_numpy(pool.hull_cnt).to(dev)
    p = torch.from_numpy(pool.pairs.reshape(-1).copy()).to(dev)
    out = torch.empty(n * 128, dtype=torch.uint8, device=dev)
    wsb = gjkepa.workspace_bytes_for(n, 0)          # 32-vertex hulls: no park slots
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(dev)

    def rate(steps=20):
        # chain_ms: each chain's own span on the GPU (its head event to its last kernel's end, from the
        # library's launch timing), which excludes any gap while the host thread was still enqueueing it
        gjkepa.launch_timing(True)
        with torch.cuda.stream(s):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t = time.perf_counter()
            e0.record(s)
            for _ in range(steps):
                gjkepa.gjkepa_batch_device(2, 1.0, gjkepa.DTYPE_F32, gjkepa.PREC_F64, v.data_ptr(), o.data_ptr(),
                                           c.data_ptr(), p.data_ptr(), n, out.data_ptr(), ws.data_ptr(), wsb,
                                           s.cuda_stream)
            e1.record(s)
            s.synchronize()
            wall = time.perf_counter() - t
        gjkepa.launch_timing(False)
        lt = gjkepa.launch_timing_read()
        chain_ms = float(np.mean([lt["end_ms"][lt["chain"] == k].max() for k in set(lt["chain"].tolist())]))
        return {"M_per_s_events": round(n * steps / (e0.elapsed_time(e1) * 1e-3) / 1e6, 2),
                "M_per_s_wall": round(n * steps / wall / 1e6, 2), "chain_ms": round(chain_ms, 4),
                "M_per_s_chain": round(n / (chain_ms * 1e-3) / 1e6, 2)}

    rng = np.random.default_rng(3)
    qs = []
    for _ in range(64):
        a = rng.normal(size=(32, 3)); a /= np.linalg.norm(a, axis=1, keepdims=True)
        b = rng.normal(size=(32, 3)); b /= np.linalg.norm(b, axis=1, keepdims=True)
        b += rng.normal(size=3) * 0.6
        qs.append((a, b))
    rate(3)
    res = {"alone": rate()}
    for T in threads:
        stop, calls = threading.Event(), []

        def traffic():
            k = 0
            while not stop.is_set():
                a, b = qs[k % len(qs)]
                gjkepa.gjkepa(2, 1.0, a, b)
                k += 1
            calls.append(k)
        th = [threading.Thread(target=traffic) for _ in range(T)]
        for x in th:
            x.start()
        time.sleep(0.2)
        t = time.perf_counter()
        r = rate()
        r["query_calls_per_s"] = None
        stop.set()
        for x in th:
            x.join()
        r["query_calls_per_s"] = round(sum(calls) / (time.perf_counter() - t + 0.2), 0)
        res[f"with_{T}_query_threads"] = r
    gjkepa.query_service_stop(-1)
    res["alone_after_stop"] = rate()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
