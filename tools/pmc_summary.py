"""Summarise rocprofv3 kernel-trace + PMC passes per kernel (HBM traffic per launch), and
check the bench's in-run HIP-event timing of its dominant kernel against the trace.

  python tools/pmc_summary.py <prof_dir> <pmc_fetch_dir> <pmc_write_dir> <out.json> [<bench_log>]

FETCH_SIZE / WRITE_SIZE are in KiB. On gfx950 FETCH_SIZE reports 1/2 of the bytes of a
wide (16 B/lane) coalesced read (MI355X_MICROARCH.md §HBM) — the GEMM operands arrive by
16-B/lane buffer_load ... lds, so FETCH is doubled for the gemm kernels (the narrower epilogue
loads are uncalibrated and counted as reported). WRITE_SIZE is taken as reported.

With <bench_log> (the JSON line bench.py printed under the same rocprofv3 run, run with
--no-breakdown --no-all-slots-rate so the dominant kernel's last steps*launches_per_step
dispatches ARE the timed region), the trace's mean duration over those dispatches is written
next to the bench's event-measured avg_launch_ms ("dominant_kernel_check").
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


def main(prof_dir, fetch_dir, write_dir, out, bench_log=None):
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
    if bench_log:
        line = [ln for ln in open(bench_log) if ln.startswith("{")][-1]
        b = json.loads(line)
        rf = b["roofline"]
        n = int(round(rf["launches_per_step"] * b["steps"]))
        trace = [r for r in _rows(prof_dir, "*kernel_trace.csv") if rf["kernel"] in r["Kernel_Name"]]
        trace.sort(key=lambda r: int(r["Start_Timestamp"]))
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in trace[-n:]]
        res["dominant_kernel_check"] = {
            "kernel": rf["kernel"], "timed_dispatches": len(durs),
            "trace_avg_ms_timed_region": sum(durs) / max(len(durs), 1) / 1e6,
            "trace_avg_ms_all_dispatches": sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in trace)
            / max(len(trace), 1) / 1e6,
            "bench_event_avg_ms": rf["avg_launch_ms"], "bench_value_under_rocprof": b["value"]}
        print(json.dumps(res["dominant_kernel_check"]))
    json.dump(res, open(out, "w"), indent=1)
    for k, v in sorted(((k, v) for k, v in res.items() if "hbm_bytes_per_launch" in v),
                       key=lambda kv: -kv[1]["hbm_bytes_per_launch"])[:12]:
        print(f'{v["hbm_bytes_per_launch"] / 1e6:10.1f} MB/launch  {k[:90]}')


if __name__ == "__main__":
    main(*sys.argv[1:6])
