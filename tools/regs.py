#!/usr/bin/env python3
"""Per-kernel register summary from hipcc -Rpass-analysis=kernel-resource-usage output on stdin: regs.py [substr]"""
import re
import sys

cur, rows = None, {}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|VGPRs Spill|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).split()[0] + ("Spill" if "Spill" in m.group(1) else "")] = int(m.group(2))
sub = sys.argv[1] if len(sys.argv) > 1 else ""
for k, v in rows.items():
    if sub in k:
        print(k[:90], v)
