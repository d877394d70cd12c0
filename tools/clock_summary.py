"""Effective clock per kernel from a GRBM_GUI_ACTIVE pass (MI355X_MICROARCH.md, DVFS give-back:
clock ~= GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time; reads high below ~0.3 ms dispatches).

  python tools/clock_summary.py <pmc_dir> <out.json>
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(d, out):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    acc = defaultdict(lambda: [0.0, 0.0, 0])
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
            continue
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        a = acc[r["Kernel_Name"]]
        a[0] += float(r["Counter_Value"]); a[1] += dur; a[2] += 1
    res = {}
    for k, (cyc, ns, n) in sorted(acc.items(), key=lambda kv: -kv[1][1]):
        if ns <= 0:
            continue
        res[k] = {"launches": n, "avg_ms": ns / n / 1e6, "effective_ghz": cyc / 8.0 / ns}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in list(res.items())[:12]:
        print(f"{v['effective_ghz']:.3f} GHz  {v['avg_ms']:.4f} ms x{v['launches']}  {k[:90]}")


if __name__ == "__main__":
    main(*sys.argv[1:3])
