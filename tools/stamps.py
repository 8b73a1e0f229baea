#!/usr/bin/env python3
"""Per-phase wave-time breakdown from a -DGJKEPA_DIAG_STAMPS build (tools/build_variant.sh stamps
-DGJKEPA_DIAG_STAMPS).  Runs one warm-up batch, clears the counters, runs one measured batch and
prints the share of summed wave time per phase.  usage: GJKEPA_LIB=<stamps .so> python
tools/stamps.py [C2|C4|C5] [n_pairs]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "collision-detect-gjk-epa_amd"))
sys.path.insert(0, ROOT)
import gjkepa  # noqa: E402
from bench import CONFIGS, SEED  # noqa: E402

NAMES = {0: "gjk.load", 1: "gjk.sphere", 2: "gjk.init", 3: "gjk.update_simplex", 4: "gjk.checks+inside",
         5: "gjk.store", 6: "gjk.route", 10: "epa.load", 11: "epa.iter1", 12: "epa.dir", 13: "epa.support",
         14: "epa.visible", 15: "epa.horizon", 16: "epa.compact", 17: "epa.cone", 18: "epa.term",
         19: "ct.nearest", 20: "ct.contact", 21: "ct.type", 22: "epa.store", 23: "epa.route",
         24: "ct.route", 25: "ct.load", 26: "ct.store"}


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
    nmin, nmax, rmax, n_default, _ = CONFIGS[cfg]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else n_default
    lib = gjkepa.load()
    lib.gjkepa_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    pool = gjkepa.synth_pairs(SEED, n, nmin, nmax, rmax, dtype=np.float32)
    buf = np.zeros(32, dtype=np.uint64)
    gjkepa.gjkepa_batch(pool, 2, 1.0, gjkepa.PREC_F64)
    lib.gjkepa_diag_stamps(buf.ctypes.data, 1)
    gjkepa.gjkepa_batch(pool, 2, 1.0, gjkepa.PREC_F64)
    lib.gjkepa_diag_stamps(buf.ctypes.data, 1)
    for lo, hi, title in ((0, 10, "GJK kernels"), (10, 32, "EPA + contact kernels")):
        tot = float(buf[lo:hi].sum())
        print(f"== {cfg} {title}: {tot / n:.0f} wave-ticks per pair")
        for i in range(lo, hi):
            if buf[i]:
                print(f"   {NAMES.get(i, i):22s} {100 * buf[i] / tot:6.2f} %  {buf[i] / n:10.1f} ticks/pair")


if __name__ == "__main__":
    main()
