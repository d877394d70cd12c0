"""The kernel sequence of ONE step from a rocprofv3 kernel-trace CSV: the launches between the
last two `adam_flat_kernel` launches (the optimizer ends every step), each with its duration and
the gap since the previous kernel ended — to attribute the short / copy kernels of a step.

  python tools/trace_seq.py <dir with *kernel_trace.csv> [--step -1] > seq.txt
"""
import re
import sys

from trace_stats import load


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"at::native::", "", name)
    return name[:110]


def main():
    rows = load(sys.argv[1])
    k = int(sys.argv[sys.argv.index("--step") + 1]) if "--step" in sys.argv else -1
    ends = [i for i, r in enumerate(rows) if "adam_flat_kernel" in r[0]]
    if len(ends) < 2:
        sys.exit("fewer than two optimizer launches in the trace")
    a, b = ends[k - 1], ends[k]
    seg = rows[a + 1:b + 1]
    prev = rows[a][2]
    tot = 0
    for i, (name, s, e) in enumerate(seg):
        print(f"{i:4d} {(e - s) / 1e3:8.2f} us  gap {(s - prev) / 1e3:6.2f}  {short(name)}")
        prev = max(prev, e)
        tot += e - s
    print(f"{len(seg)} kernels, {tot / 1e6:.3f} ms busy, {(seg[-1][2] - rows[a][2]) / 1e6:.3f} ms wall")


if __name__ == "__main__":
    main()
