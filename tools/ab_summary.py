"""Summarise an A/B log of tools/ab_lib_gemm.sh: per shape and variant, the A and B rates of each run.
  python tools/ab_summary.py gpurun_out/ab.log [variant ...]"""
import ast
import collections
import re
import sys

R = collections.defaultdict(lambda: collections.defaultdict(list))
cur = None
for line in open(sys.argv[1]):
    if line.startswith("=="):
        cur = line.split()[1]
        continue
    m = re.match(r"(.*?) (\{.*\})$", line.strip())
    if m and cur:
        for k, v in ast.literal_eval(m.group(2)).items():
            R[m.group(1)][(cur, k)].append(v)
keys = sys.argv[2:]
for shape, dd in R.items():
    ks = keys or sorted({k for _, k in dd})
    print(shape)
    for k in ks:
        a, b = dd[("A", k)], dd[("B", k)]
        if a and b:
            print(f"   {k:14s} A {a}  B {b}  A/B {sum(a) / sum(b):.3f}")
