#!/usr/bin/env python3
"""Print the headline fields of a bench line (or, with --ab DIR, the A/B lines of tools/gpu_session.sh step ab)."""
import glob
import json
import os
import sys


def line(p):
    return json.loads([x for x in open(p) if x.startswith("{")][-1])


def brief(d):
    dk = d.get("dominant_kernel") or {}
    s = {"value": d["value"], "ms": d["ms_per_step"], "dom": dk.get("kernel"), "dom_frac": dk.get("frac"),
         "dom_launch_ms": dk.get("launch_ms"), "span_ms": dk.get("wall_span_ms"), "parity": (d.get("parity_sample") or {}).get("all_equal")}
    for c, l in (d.get("legs") or {}).items():
        s[c] = {"value": l["value"], "chain_ms": l["chain_ms"], "dom": l["dominant_kernel"]["kernel"],
                "frac": l["dominant_kernel"]["frac"], "parity": (l.get("parity_sample") or {}).get("all_equal")}
    if "fp32_compute" in d:
        s["fp32"] = {k: d["fp32_compute"].get(k) for k in ("value", "gate_passed", "depth_err_over_max1d_max")}
    return s


if __name__ == "__main__":
    if sys.argv[1] == "--ab":
        for p in sorted(glob.glob(os.path.join(sys.argv[2], "ab_*.json"))):
            print(os.path.basename(p), json.dumps(brief(line(p))))
    else:
        print(json.dumps(brief(line(sys.argv[1])), indent=1))
