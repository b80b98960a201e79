#!/usr/bin/env python3
"""Per-kernel VGPR / AGPR / spill / occupancy table from hipcc's
-Rpass-analysis=kernel-resource-usage remarks (stdin), filtered by a
substring of the mangled name:
    hipcc ... --cuda-device-only -c x.hip -o /dev/null \\
        -Rpass-analysis=kernel-resource-usage 2>&1 | python3 tools/resource_usage.py k_aead_tile"""
import re
import sys

pat = sys.argv[1] if len(sys.argv) > 1 else ""
cur, rows = None, []
for line in sys.stdin:
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = int(m.group(2))
for r in rows:
    if pat in r["name"]:
        print("%-80s VGPR %3s AGPR %3s spillV %3s spillS %3s occ %s LDS %s" % (
            r["name"][:80], r.get("VGPRs"), r.get("AGPRs"), r.get("VGPRs Spill"), r.get("SGPRs Spill"),
            r.get("Occupancy"), r.get("LDS Size")))
