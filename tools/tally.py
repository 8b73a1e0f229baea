#!/usr/bin/env python3
"""GPU box: pairs routed to every route code in one chain (the workspace's tallies) and park slots taken,
for a config's full batch.  usage: python tools/tally.py C2 C4 C5"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "collision-detect-gjk-epa_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gjkepa  # noqa: E402
from bench import CONFIGS, SEED  # noqa: E402

NAMES = {1: "GJK1", 2: "GJK2"}
NAMES.update({0x10 + t: f"EPA{t}" for t in range(6)})
NAMES.update({0x20 + c: f"CT{c // 2}.{c % 2}" for c in range(12)})
NAMES[0x2E] = "REDO"
for cfg in sys.argv[1:] or ["C2", "C4", "C5"]:
    nmin, nmax, rmax, n, _ = CONFIGS[cfg]
    pool = gjkepa.synth_pairs(SEED, n, nmin, nmax, rmax)
    dev = torch.device("cuda", 0)
    t = {k: torch.from_numpy(v).to(dev) for k, v in (("v", pool.verts), ("o", pool.hull_off), ("c", pool.hull_cnt),
                                                      ("p", pool.pairs.reshape(-1).copy()))}
    for prec in (gjkepa.PREC_F64, gjkepa.PREC_F32):
        out = torch.empty(n * gjkepa.load().gjkepa_record_bytes(prec), dtype=torch.uint8, device=dev)
        wsb = gjkepa.workspace_bytes_for(n, gjkepa.large_pairs(pool))     # as bench.py sizes it
        ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
        gjkepa.gjkepa_batch_device(2, 1.0, gjkepa.DTYPE_F32, prec, t["v"].data_ptr(), t["o"].data_ptr(), t["c"].data_ptr(),
                                   t["p"].data_ptr(), n, out.data_ptr(), ws.data_ptr(), wsb, 0)
        torch.cuda.synchronize()
        h = ws[:512].cpu().numpy().view(np.uint32)
        tally = h[gjkepa.WS_COUNTERS:gjkepa.WS_COUNTERS + gjkepa.WS_TALLY]
        parts = {NAMES.get(k, hex(k)): int(v) for k, v in enumerate(tally) if v}
        print(cfg, "fp64" if prec == gjkepa.PREC_F64 else "fp32", "routed:", parts, "park slots taken:", int(h[gjkepa.WS_PARK_WORD]),
              flush=True)
