"""Micro-benchmark of the NN (chamfer) kernels: Gpair-dist/s on the SURVEY §8(d) shapes.

  python tools/nn_bench.py [--iters 50]
Unique pairs per call = B*n*m (both directions come from the same pair set).
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

ge.add_pkg_path()
from ured_hip import nn as unn  # noqa: E402


def timeit(fn, iters, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    res = {}
    for (B, n, m) in [(16, 2048, 2048), (64, 4096, 4096), (32, 2000, 1000), (16, 4096, 2048), (16, 16384, 2048), (4096, 1024, 1024)]:
        p1 = torch.rand(B, n, 3, generator=g).to(dev)
        p2 = torch.rand(B, m, 3, generator=g).to(dev)
        t_f = timeit(lambda: unn.nn_dense(p1, p2), a.iters)
        unn.FUSED = False
        t_2p = timeit(lambda: unn.nn_dense(p1, p2), a.iters)
        unn.FUSED = True
        q1 = p1.clone().requires_grad_(True)

        def fb():
            d1, d2, _, _ = unn.nn_dense(q1, p2)
            d1.sum().backward()
        t_fb = timeit(fb, a.iters)
        pairs = B * n * m
        res[f"{B}x{n}x{m}"] = {"fwd_ms": t_f * 1e3, "fwd_gpair_s": pairs / t_f / 1e9,
                               "two_pass_fwd_ms": t_2p * 1e3, "two_pass_gpair_s": pairs / t_2p / 1e9,
                               "fwdbwd_ms": t_fb * 1e3, "fwdbwd_gpair_s": pairs / t_fb / 1e9}
        print(f"{B}x{n}x{m}: fwd {t_f*1e3:.3f} ms ({pairs/t_f/1e9:.1f} Gpair/s; two-pass {pairs/t_2p/1e9:.1f})  fwd+bwd {t_fb*1e3:.3f} ms ({pairs/t_fb/1e9:.1f} Gpair/s)", flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
