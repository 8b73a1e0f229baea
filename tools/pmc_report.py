#!/usr/bin/env python3
"""Per-launch-chain PMC summary of a PMC run (tools/gpu_session.sh step pmc), for bench.py's roofline fields.

Every kernel of the GJK/EPA/contact chain is dispatched once per bench step; counters are
averaged over a kernel's dispatches and summed over the chain.  HBM traffic follows
/opt/skills/guides/MI355X_MICROARCH.md (§HBM): FETCH_SIZE and WRITE_SIZE are KiB, and on gfx950
FETCH_SIZE counts half the bytes of wide reads, so traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
VALU issue: SQ_INSTS_VALU wave-instructions; `valu_issue_frac` prices each at the 2-cycle wave64
issue slot (32 lanes/clock) against 1024 SIMDs x the chain's kernel time x 2.4 GHz (fp64 ops take
longer, so this is a lower bound on VALU-pipe occupancy).
The entry carries the library source hash the passes ran (gjkepa_version_string); bench.py uses
it only when the loaded library has the same hash.
usage: python tools/pmc_report.py <dir> <key> <n_pairs>  (merges into profiles/pmc_traffic.json); <dir> holds
the passes p1..p5 (tools/gpu_session.sh step pmc: gpurun_out/<tag>/pmc_<config>)"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag, key, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
    base = tag if os.path.isdir(tag) else os.path.join(ROOT, "gpurun_out", tag, "pmc")
    per = collections.defaultdict(lambda: collections.defaultdict(dict))
    dur = collections.defaultdict(dict)
    for f in sorted(glob.glob(f"{base}/p*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if "gk::" not in k or (k.startswith("gk::gjk_kernel") and k.endswith(", true>")):   # warm-start GJK: not the chain
                continue
            d = per[k][r["Counter_Name"]]
            d[r["Dispatch_Id"]] = d.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    for f in sorted(glob.glob(f"{base}/p*/run_kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if "gk::" not in k or (k.startswith("gk::gjk_kernel") and k.endswith(", true>")):   # warm-start GJK: not the chain
                continue
            dur[k][f + r.get("Dispatch_Id", "")] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    # one chain = one dispatch of GJK tier 0 (it takes every pair); a kernel dispatched several times
    # per chain (the contact tiers, once per EPA tier's contact pass) is summed over its dispatches
    g0 = [k for k in per if k.startswith("gk::gjk_kernel") and k.split(",")[2].strip() == "4"]
    nchain = {c: len(v) for c, v in per[g0[0]].items()} if g0 else {}
    kernels = {}
    for k, cs in per.items():
        kernels[k] = {c: sum(v.values()) / max(nchain.get(c, len(v)), 1) for c, v in cs.items()}
        if dur.get(k):
            n_g0 = len(dur[g0[0]]) if g0 and dur.get(g0[0]) else len(dur[k])
            kernels[k]["seconds"] = sum(dur[k].values()) / max(n_g0, 1)
            kernels[k]["dispatches_per_chain"] = len(dur[k]) / max(n_g0, 1)
    tot = collections.Counter()
    for m in kernels.values():
        tot.update(m)
    traffic = (2.0 * tot["FETCH_SIZE"] + tot["WRITE_SIZE"]) * 1024.0
    secs = tot["seconds"]
    srcs = set()
    for f in sorted(glob.glob(f"{base}/p*.json")):
        for line in open(f):
            if line.startswith("{"):
                srcs.add(json.loads(line)["lib"].rsplit("src ", 1)[-1].strip())
    if len(srcs) != 1:
        sys.exit(f"PMC passes disagree on (or lack) the library source hash: {srcs}")
    entry = {
        "src": srcs.pop(),
        "bytes_per_launch": traffic,
        "fetch_bytes_raw": tot["FETCH_SIZE"] * 1024.0,
        "fetch_bytes_corrected": 2.0 * tot["FETCH_SIZE"] * 1024.0,
        "fetch_correction": "x2, calibrated on this access shape: profiles/r03/fetch_calib.json (4-B/lane "
                            "coalesced reads and the GJK tier-0 hull-load pattern both read 2.0 / 1.97 bytes per "
                            "FETCH_SIZE byte, like the guide's 16-B/lane case)",
        "write_bytes": tot["WRITE_SIZE"] * 1024.0,
        "valu_instr": tot["SQ_INSTS_VALU"],
        "valu_instr_per_query": tot["SQ_INSTS_VALU"] / n,
        "chain_kernel_seconds": secs,
        "valu_issue_frac": tot["SQ_INSTS_VALU"] * 2.0 / (1024 * secs * 2.4e9) if secs else None,
        # SQ_ACTIVE_INST_VALU counts quad-cycles (MI355X_MICROARCH.md, cycle constants): x4 = cycles in
        # which a wave had a VALU instruction issuing; against 1024 SIMDs x kernel time x 2.4 GHz
        "valu_busy_frac": tot["SQ_ACTIVE_INST_VALU"] * 4.0 / (1024 * secs * 2.4e9) if secs and tot["SQ_ACTIVE_INST_VALU"] else None,
        "kernels": kernels,
        "source": f"tools/gpu_session.sh pmc run {tag}, kernels summed over their dispatches per chain (one chain = one GJK tier-0 dispatch), summed over the chain",
    }
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    allj = json.load(open(path)) if os.path.exists(path) else {}
    allj[key] = entry
    json.dump(allj, open(path, "w"), indent=1)
    print(json.dumps({k: v for k, v in entry.items() if k != "kernels"}, indent=1))


if __name__ == "__main__":
    main()
