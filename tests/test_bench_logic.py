"""CPU tests of bench.py's roofline logic (no GPU): the dominant kernel is the one with the most launch
time per chain; its wall span is the union of its launches' intervals (two concurrent parts count
once); the pairs a parted launch serves are its route code's tally split by the hits in its range;
achieved = pairs per launch x bytes per pair / mean launch duration."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import gjkepa  # noqa: E402


def _rec(kernel, tier, chain, start, end, first=0, n=0, code=-1, part=0, stream=0):
    r = np.zeros(1, gjkepa.LAUNCH_TIME)
    r["kernel"], r["tier"], r["chain"], r["start_ms"], r["end_ms"] = kernel, tier, chain, start, end
    r["first_pair"], r["n_pairs"], r["route_code"], r["part"], r["stream"] = first, n, code, part, stream
    return r


def _chain(c, n):
    return [
        _rec(b"gjk", 0, c, 0.0, 1.0, 0, n),
        _rec(b"epa", 0, c, 1.0, 4.0, 0, n // 2, bench.ROUTE_EPA0, 0, 0),
        _rec(b"epa", 0, c, 1.1, 5.5, n // 2, n - n // 2, bench.ROUTE_EPA0, 1, 1),
        _rec(b"contact", 0, c, 4.0, 6.0, 0, n // 2, bench.ROUTE_CT0, 0, 2),   # 2.0 ms, but less than EPA's 7.4
        _rec(b"contact", 0, c, 6.0, 6.5, n // 2, n - n // 2, bench.ROUTE_CT0, 1, 2),
    ]


def test_busy_span_is_the_union_of_intervals():
    rs = np.concatenate([_rec(b"epa", 0, 0, 1.0, 4.0), _rec(b"epa", 0, 0, 1.1, 5.5), _rec(b"epa", 0, 0, 7.0, 8.0)])
    assert abs(bench.busy_span(rs) - (4.5 + 1.0)) < 1e-6


def test_dominant_kernel_parts_and_pairs():
    n = 1000
    lt = np.concatenate(_chain(0, n) + _chain(1, n))
    tally = np.zeros(bench.WS_TALLY, np.uint32)
    tally[bench.ROUTE_EPA0] = 600
    recs = np.zeros(n, gjkepa.REC64)
    recs["collision"][:400] = 1           # 400 hits in the first half, 200 in the second
    recs["collision"][500:700] = 1
    d = bench.dominant_kernel(lt, tally, recs, 928.0, None)
    assert d["kernel"] == "epa tier 0" and d["launches_per_step"] == 2.0
    assert abs(d["wall_span_ms"] - 4.5) < 1e-6                        # union of [1, 4] and [1.1, 5.5]
    assert abs(d["pairs_per_step"] - 600) < 1e-6 and abs(d["pairs_per_launch"] - 300) < 1e-6
    launch_ms = (3.0 + 4.4) / 2
    assert abs(d["launch_ms"] - launch_ms) < 1e-4
    assert abs(d["achieved"] - 300 * 928.0 / (launch_ms * 1e-3) / 1e9) < 1e-3
    assert abs(d["span_achieved"] - 600 * 928.0 / 4.5e-3 / 1e9) < 1e-3
    assert d["frac"] == round(d["achieved"] / bench.PEAK_HBM_GBS, 6)
