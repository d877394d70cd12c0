"""Per-kernel VGPR / spill / occupancy table from hipcc -Rpass-analysis=kernel-resource-usage output
(stdin). Usage: hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python tools/kres.py [filter]"""
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
    m = re.search(r"remark:\s+([A-Za-z \[\]/]+?):\s*(\S+)\s*\[", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
for k, v in rows.items():
    if flt in k:
        print(f"{v.get('VGPRs','?'):>4} vgpr {v.get('VGPRs Spill','?'):>3} vspill {v.get('SGPRs Spill','?'):>3} sspill "
              f"occ {v.get('Occupancy [waves/SIMD]','?')}  {k}")
