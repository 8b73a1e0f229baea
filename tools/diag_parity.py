"""Diagnostic: GPU kernels vs oracle on small seeded sets of every config; prints mismatches."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "collision-detect-gjk-epa_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np
import gjkepa, oracle, parity

cube = np.array([[x, y, z] for z in (0, 1) for y in (0, 1) for x in (0, 1)], float)
offs = [(0.5, 0.2, 0.1), (1, 0, 0), (1 + 1e-9, 0, 0), (0, 0, 1e-3), (0.5, 0.5, 0.1), (0.3, 0.2, 0.1), (0.9, 0.8, 0.7), (0.9, 0.25, 0), (3, 0, 0), (0, 0, 0), (0.3, 0.3, 0.3), (1, 1, 1)]
pool = gjkepa.HullPool.from_pairs([(cube, cube + np.array(o)) for o in offs])
for v in (1, 2, 3):
    g = gjkepa.gjkepa_batch(pool, v, 1e-3)
    r = oracle.gjkepa_batch(pool, v, 1e-3)
    c = parity.compare(g, r)
    print("cubes v%d" % v, {k: c[k] for k in c if k != "bad_idx"}, flush=True)
    for i in c["bad_idx"][:5]:
        print("  off", offs[i], "\n   gpu", parity.fmt(g[i]), "\n   ref", parity.fmt(r[i]))
cfgs = {"C2": (32, 32, 2.5, 20000), "C4": (8, 256, 2.5, 3000), "C5": (32, 128, 0.3, 3000)}
for name, (a, b, rm, n) in cfgs.items():
    pool = gjkepa.synth_pairs(0x6A4B5C1D, n, a, b, rm)
    for v in (2, 1, 3):
        t = time.time(); g = gjkepa.gjkepa_batch(pool, v, 1.0); tg = time.time() - t
        t = time.time(); r = oracle.gjkepa_batch(pool, v, 1.0); tr = time.time() - t
        c = parity.compare(g, r)
        print(name, "v%d" % v, "gpu %.3fs cpu %.3fs" % (tg, tr), {k: c[k] for k in c if k != "bad_idx"}, flush=True)
        for i in c["bad_idx"][:4]:
            print("  pair", i, "\n   gpu", parity.fmt(g[i]), "\n   ref", parity.fmt(r[i]))
    gf = gjkepa.gjkepa_batch(pool, 2, 1.0, precision=gjkepa.PREC_F32)
    r = oracle.gjkepa_batch(pool, 2, 1.0)
    c = parity.compare(gf, r, rtol=1e-3, atol=1e-5)
    print(name, "fp32 compute", {k: c[k] for k in c if k != "bad_idx"}, flush=True)
