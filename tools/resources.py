"""Per-kernel register / scratch / occupancy table from hipcc -Rpass-analysis=kernel-resource-usage
output (stdin).  usage: hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python3 tools/resources.py [filter]"""
import re
import sys

cur, rows = None, []
for line in sys.stdin:
    m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", line)
    if not m:
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
flt = sys.argv[1] if len(sys.argv) > 1 else ""
for r in rows:
    if flt in r["name"]:
        print(f"{r['name'][:70]:70s} VGPR {r.get('VGPRs','?'):>4} AGPR {r.get('AGPRs','?'):>3} "
              f"SGPRspill {r.get('SGPRs Spill','?'):>4} VGPRspill {r.get('VGPRs Spill','?'):>3} "
              f"scratch {r.get('ScratchSize [bytes/lane]','?'):>3} occ {r.get('Occupancy [waves/SIMD]','?')}")
