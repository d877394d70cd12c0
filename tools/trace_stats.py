"""Per-kernel statistics from a rocprofv3 kernel-trace CSV (what --stats prints, computed here
so that a trace-only run — no --stats — can be summarised too), optionally restricted to the
kernels launched between the first and last launch of a marker kernel.

  python tools/trace_stats.py <dir with *kernel_trace.csv> [out.csv] [--top 40] [--exclusive] [--tail K/T]
  (--tail K/T: per kernel, only the last K/T of its launches — the bench's K timed steps of T)
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort(key=lambda t: t[1])
    return rows


def tail(rows, frac):
    """Per kernel name, keep the last round(n * frac) launches (e.g. the bench's timed steps:
    frac = steps / (warmup + 1 + steps), every step launching the same kernels)."""
    by = defaultdict(list)
    for r in rows:
        by[r[0]].append(r)
    keep = []
    for name, rs in by.items():
        k = max(1, int(round(len(rs) * frac)))
        keep += rs[-k:]
    keep.sort(key=lambda t: t[1])
    return keep


def stats(rows, exclusive=False):
    """exclusive: a kernel's time counted from max(its start, the previous kernel's end) — the
    part of its duration not overlapped with its predecessor's tail (kernels of one stream may
    start while the previous one drains when the dispatch carries no barrier)."""
    by = defaultdict(list)
    prev_end = None
    for name, s, e in rows:
        s0 = max(s, prev_end) if (exclusive and prev_end is not None) else s
        by[name].append(max(e - s0, 0))
        prev_end = e if prev_end is None else max(prev_end, e)
    out = []
    for name, ds in by.items():
        out.append((name, len(ds), sum(ds), sum(ds) / len(ds), min(ds), max(ds)))
    out.sort(key=lambda t: -t[2])
    return out


def main():
    d = sys.argv[1]
    dst = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else None
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
    rows = load(d)
    if "--tail" in sys.argv:
        a, b = sys.argv[sys.argv.index("--tail") + 1].split("/")
        rows = tail(rows, int(a) / int(b))
    st = stats(rows, exclusive="--exclusive" in sys.argv)
    tot = sum(t[2] for t in st)
    if dst:
        with open(dst, "w") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
            for name, n, s, a, mn, mx in st:
                w.writerow([name, n, s, round(a, 1), mn, mx, round(100.0 * s / max(tot, 1), 4)])
    for name, n, s, a, mn, mx in st[:top]:
        print(f"{n:7d} {s / 1e6:10.3f} ms {a / 1e3:9.2f} us  {name[:110]}")


if __name__ == "__main__":
    main()
