"""Print the per-step kernel table of a rocprofv3 kernel_stats.csv (bench: steps+warmup launches)."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 23
pat = sys.argv[3:] 
rows = list(csv.DictReader(open(path)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total {tot / steps / 1e6:.3f} ms/step")
sel = [r for r in rows if any(p in r['Name'] for p in pat)] if pat else \
    sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:30]
for r in sel:
    print(f"{float(r['TotalDurationNs']) / steps / 1e3:8.1f} us {int(r['Calls']) / steps:6.1f}x "
          f"{float(r['AverageNs']) / 1e3:7.1f}  {r['Name'][:110]}")
