#!/usr/bin/env python3
"""Timeline of the last narrow-phase chain in a rocprofv3 kernel trace (run_kernel_trace.csv):
start / end / duration (us, relative to the chain's first kernel), queue and kernel.
usage: python3 tools/trace_chain.py <run_kernel_trace.csv> [n_chains_back]"""
import csv
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    back = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    heads = [i for i, r in enumerate(rows) if "ws_reset" in r["Kernel_Name"] or "fillBuffer" in r["Kernel_Name"]]
    if not heads:
        sys.exit("no chain head (ws_reset_kernel) in the trace")
    i0 = heads[-back]
    i1 = heads[-back + 1] if back > 1 else len(rows)
    chain = [r for r in rows[i0:i1] if "gk::" in r["Kernel_Name"]]
    t0 = int(chain[0]["Start_Timestamp"])
    end = 0
    for r in chain:
        s = (int(r["Start_Timestamp"]) - t0) / 1e3
        e = (int(r["End_Timestamp"]) - t0) / 1e3
        end = max(end, e)
        name = r["Kernel_Name"].replace("void gk::", "").split("(")[0]
        print(f"{s:9.1f} {e:9.1f} {e - s:8.1f}  q{r['Queue_Id']} grid {int(r['Grid_Size_X']) // 64:6d}  {name[:80]}")
    print(f"chain: {end:.1f} us over {len(chain)} launches")


if __name__ == "__main__":
    main()
