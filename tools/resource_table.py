#!/usr/bin/env python3
"""Condense `make resource-usage` (hipcc -Rpass-analysis=kernel-resource-usage)
into one row per kernel instantiation: VGPR / AGPR / SGPR / LDS / scratch /
occupancy.  Usage: make resource-usage 2>&1 | python tools/resource_table.py"""
import re
import subprocess
import sys

rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"remark:\s+Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+([A-Za-z \[\]/]+?):\s*(-?\d+)", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = int(m.group(2))


def demangle(n):
    try:
        return subprocess.run(["c++filt", n], capture_output=True, text=True).stdout.strip()
    except OSError:
        return n


cols = ["VGPRs", "AGPRs", "TotalSGPRs", "LDS Size [bytes/block]", "ScratchSize [bytes/lane]",
        "Occupancy [waves/SIMD]"]
print("kernel | VGPR | AGPR | SGPR | LDS B/block | scratch B/lane | waves/SIMD")
print("---|---|---|---|---|---|---")
for r in rows:
    name = demangle(r["name"]).replace("void dtc::", "").replace("(dtc::PassArgs)", "")
    print(name + " | " + " | ".join(str(r.get(c, "")) for c in cols))
