#!/usr/bin/env python3
"""hipcc -Rpass-analysis=kernel-resource-usage output (stdin) -> one line per kernel:
VGPRs, VGPR spills, scratch bytes/lane, occupancy.  usage:
  hipcc ... -Rpass-analysis=kernel-resource-usage -c f.hip -o /dev/null 2>&1 | tools/kres.py [filter]"""
import re
import sys

flt = sys.argv[1] if len(sys.argv) > 1 else ""
cur, rows = None, {}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[bytes/lane\]| \[waves/SIMD\]|)\s*:\s*(\S+)", line)
    if cur and m:
        rows[cur][m.group(1).strip()] = m.group(2)
for k, v in rows.items():
    if flt in k:
        print(f"{v.get('VGPRs','?'):>4} vgpr  spill {v.get('VGPRs Spill','?'):>3}  scratch {v.get('ScratchSize','?'):>4}  "
              f"occ {v.get('Occupancy','?')}  {k}")
