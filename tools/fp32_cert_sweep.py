#!/usr/bin/env python3
"""CPU: the fp32 certificate's thresholds against the full-batch gate, without a GPU.

The GPU's fp32 records are byte-identical to a CPU model of the fp32 path (tools/fp32_check.py: the
fp32 build of the oracle, with the pairs its certificate flags replaced by the fp64 records).  This
sweeps the model's certificate thresholds (oracle_cert_drop / oracle_cert_gap: the float globals of
libgjkepa_oracle_f32.so, the same values as csrc/gk_common.h Tol<float>::CERT_*) and reports, per
config and threshold, the pairs sent to the fp64 redo and the gate metrics of tools/fp32_metrics.py at
the gate's normal bound.  Swept: the noise allowance, k x 2^-24 x (|A| + |B|), added to the support gap.  usage: python tools/fp32_cert_sweep.py [C2 C5 C4] [--pairs N]
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "collision-detect-gjk-epa_amd"), os.path.join(ROOT, "oracle"), ROOT,
                os.path.join(ROOT, "tools")]

import numpy as np  # noqa: E402

import gjkepa  # noqa: E402
import oracle  # noqa: E402
from bench import CONFIGS, SEED, host_cpus  # noqa: E402
from fp32_check import model_fp32  # noqa: E402
from fp32_metrics import fp32_report  # noqa: E402


def set_cert(gap: float, drop: float, noise: float) -> None:
    oracle.gjkepa_batch_f32(gjkepa.HullPool(np.zeros(0, np.float32), np.zeros(0, np.int64), np.zeros(0, np.int32),
                                            np.zeros((0, 2), np.int32)))          # loads the f32 library
    lib = oracle._lib32
    ctypes.c_float.in_dll(lib, "oracle_cert_gap").value = gap
    ctypes.c_float.in_dll(lib, "oracle_cert_drop").value = drop
    ctypes.c_float.in_dll(lib, "oracle_cert_noise").value = noise


def main():
    cfgs = [a for a in sys.argv[1:] if a.startswith("C")] or ["C2", "C5", "C4"]
    npairs = int(sys.argv[sys.argv.index("--pairs") + 1]) if "--pairs" in sys.argv else 0
    threads = host_cpus()["usable"]
    for cfg in cfgs:
        nmin, nmax, rmax, n, _ = CONFIGS[cfg]
        n = npairs or n
        pool = gjkepa.synth_pairs(SEED, n, nmin, nmax, rmax, dtype=np.float32)
        r64 = oracle.gjkepa_batch(pool, 2, 1.0, threads)
        for thr, k in ((5e-7, 0), (5e-7, 2), (5e-7, 4), (5e-7, 8)):
            set_cert(thr, thr, k * 2.0 ** -24)
            m, redo = model_fp32(pool, r64, threads)
            rep = fp32_report(pool, m, r64)
            rep.pop("gate", None)
            print(json.dumps({"config": cfg, "pairs": n, "cert": thr, "noise_ulps": k, "redo": int(redo.sum()),
                              "redo_frac": round(float(redo.mean()), 4), **rep}), flush=True)


if __name__ == "__main__":
    main()
