"""Summarise an A/B log of tools/ab_lib_gemm.sh: per shape and variant, the rates of each library
(A = in-tree, B, C, ... = the URED_LIB builds) and each one's ratio to A.
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
    tags = sorted({t for t, _ in dd})
    for k in ks:
        a = dd[("A", k)]
        if not a:
            continue
        row = f"   {k:14s} A {a}"
        for t in tags[1:]:
            b = dd[(t, k)]
            if b:
                row += f"  {t} {b} {t}/A {sum(b) / sum(a):.3f}"
        print(row)
