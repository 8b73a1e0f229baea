"""Summarise rocprofv3 --pmc passes for the dominant kernel (tier 0) per dispatch."""
import csv, glob, json, os, sys
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
key = sys.argv[2] if len(sys.argv) > 2 else "1, 64, 128"
base = f"gpurun_out/{tag}/pmc"
vals = {}
for f in sorted(glob.glob(f"{base}/p*/run_counter_collection.csv")):
    per = {}
    for r in csv.DictReader(open(f)):
        if key not in r["Kernel_Name"]:
            continue
        d = r["Dispatch_Id"]
        per.setdefault(r["Counter_Name"], {}).setdefault(d, 0.0)
        per[r["Counter_Name"]][d] += float(r["Counter_Value"])
    for c, dd in per.items():
        vs = list(dd.values())
        vals[c] = sum(vs) / len(vs)     # mean per dispatch
for k in sorted(vals):
    print(f"{k:28s} {vals[k]:.6g}")
json.dump(vals, open(f"{base}/summary.json", "w"), indent=1)
