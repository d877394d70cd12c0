"""The reference-API chamfer call of bench.py (chamfer_published_cmp: chamfer_3DDist forward +
backward of d1.mean() + d2.mean() at 32x2000x1000) run N times, for a rocprofv3 kernel trace:
summed kernel time per call (trace) vs the call's wall time per iteration (printed here).

  rocprofv3 --kernel-trace --stats -d gpurun_out/x -o x -- python3 tools/chamfer_api_trace.py --iters 200
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

ge.add_pkg_path()
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    r = bench.chamfer_published_cmp(torch.device("cuda:0"), iters=a.iters)
    r["calls_total"] = a.iters + 5          # + the function's 5 warm-up calls
    print(json.dumps(r), flush=True)
