#!/usr/bin/env python3
"""Compact per-kernel register / occupancy table from hipcc -Rpass-analysis=kernel-resource-usage
output (stdin).  usage: hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python tools/regs.py"""
import re
import subprocess
import sys

cur, rows = None, []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
        cur = {"name": name.replace("gk::", "").replace("(gjkepa_gjk_args)", "").replace("(gjkepa_epa_args)", "")}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|SGPRs Spill|VGPRs Spill): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1)] = int(m.group(2))
for r in rows:
    print(f"{r['name'][:70]:70s} V{r.get('VGPRs',0):4d} A{r.get('AGPRs',0):4d} scratch{r.get('ScratchSize [bytes/lane]',0):5d} "
          f"occ{r.get('Occupancy [waves/SIMD]',0):2d} sgpr_spill{r.get('SGPRs Spill',0):4d} vgpr_spill{r.get('VGPRs Spill',0):4d}")
