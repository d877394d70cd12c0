"""Summarise rocprofv3 kernel-trace + PMC passes per kernel (HBM traffic per launch).

  python tools/pmc_summary.py <prof_dir> <pmc_fetch_dir> <pmc_write_dir> <out.json>

FETCH_SIZE / WRITE_SIZE are in KiB. On gfx950 FETCH_SIZE reports 1/2 of the bytes of a
wide (16 B/lane) coalesced read (MI355X_MICROARCH.md §HBM) — the GEMM operands arrive by
16-B/lane global_load_lds, so FETCH is doubled for the gemm kernels (the narrower epilogue
loads are uncalibrated and counted as reported). WRITE_SIZE is taken as reported.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def _rows(d, pattern):
    f = glob.glob(os.path.join(d, pattern))
    return list(csv.DictReader(open(f[0]))) if f else []


def main(prof_dir, fetch_dir, write_dir, out):
    stats = {r["Name"]: r for r in _rows(prof_dir, "*kernel_stats.csv")}
    counters = defaultdict(lambda: defaultdict(list))
    for d, name in ((fetch_dir, "FETCH_SIZE"), (write_dir, "WRITE_SIZE")):
        for r in _rows(d, "*counter_collection.csv"):
            if r["Counter_Name"] == name:
                counters[r["Kernel_Name"]][name].append(float(r["Counter_Value"]))
    res = {}
    for kname, c in counters.items():
        if "gemm" not in kname and "nn_" not in kname and "bn_" not in kname and "colsum" not in kname:
            continue
        fetch = sum(c["FETCH_SIZE"]) / max(len(c["FETCH_SIZE"]), 1) * 1024.0
        write = sum(c["WRITE_SIZE"]) / max(len(c["WRITE_SIZE"]), 1) * 1024.0
        wide = "gemm" in kname
        st = stats.get(kname, {})
        res[kname] = {"launches_profiled": len(c["FETCH_SIZE"]),
                      "fetch_bytes_per_launch": fetch * (2.0 if wide else 1.0),
                      "write_bytes_per_launch": write,
                      "hbm_bytes_per_launch": fetch * (2.0 if wide else 1.0) + write,
                      "fetch_correction": "x2 (16B/lane gfx950)" if wide else "none",
                      "avg_duration_ns": float(st["AverageNs"]) if st else None}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"])[:12]:
        print(f'{v["hbm_bytes_per_launch"] / 1e6:10.1f} MB/launch  {k[:90]}')


if __name__ == "__main__":
    main(*sys.argv[1:5])
