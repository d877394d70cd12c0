"""Per-kernel SQ counter averages from one rocprofv3 --pmc pass (top kernels by time).

  python tools/sq_summary.py <pmc_dir> <out.json> [name-filter ...]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(d, out, *pat):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    val = defaultdict(lambda: defaultdict(float))
    dur, seen = defaultdict(float), defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if pat and not any(p in k for p in pat):
            continue
        val[k][r["Counter_Name"]] += float(r["Counter_Value"])
        did = r.get("Dispatch_Id", r.get("Correlation_Id"))
        if did not in seen[k]:
            seen[k].add(did)
            dur[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    res = {}
    for k in sorted(val, key=lambda k: -dur[k])[:16]:
        n = len(seen[k])
        res[k] = {"launches": n, "avg_ms": dur[k] / n / 1e6, **{c: v / n for c, v in val[k].items()}}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res.items():
        print(k[:100])
        print("   ", {c: (round(x, 4) if isinstance(x, float) else x) for c, x in v.items()})


if __name__ == "__main__":
    main(*sys.argv[1:])
