"""Config-3 inference rate alone (bench.inference_rate), plus GPU-busy vs wall time.

  python tools/infer_bench.py [--iters 30]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402
ge.add_pkg_path()
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    import bench
    from train_utils.load_sources import load_sources

    class Args:
        batch, points, parts, sources = 16, 2048, 4, 512
    cfg = bench.workload_cfg(Args)
    dev = torch.device("cuda:0")
    db, _ = load_sources(cfg, dev)
    torch.backends.cuda.preferred_blas_library("cublas")     # as bench.py --blas rocblas
    for _ in range(2):
        print(bench.inference_rate(cfg, db, dev, iters=a.iters), flush=True)


if __name__ == "__main__":
    main()
