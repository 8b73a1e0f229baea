"""Diagnostic: which axis-reject edge cases differ from the oracle (GJKEPA_LIB selects the library)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "collision-detect-gjk-epa_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np
import gjkepa, oracle, parity
import test_axis_reject as t
cs = t.cases()
pool = gjkepa.HullPool.from_pairs(cs)
g = gjkepa.gjkepa_batch(pool, 2, 1.0)
r = oracle.gjkepa_batch(pool, 2, 1.0)
bad = [i for i in range(len(r)) if g[i].tobytes() != r[i].tobytes()]
print("lib", os.environ.get("GJKEPA_LIB", "default"), "mismatches", len(bad), "of", len(r))
for i in bad[:12]:
    print(" case", i, "\n   gpu", parity.fmt(g[i]), g[i]["diag"], "\n   ref", parity.fmt(r[i]), r[i]["diag"])
