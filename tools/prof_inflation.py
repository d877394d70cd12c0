"""Does rocprofv3's kernel trace lengthen kernels? Runs the step's dominant GEMM variant (dgrad
with the BN-backward epilogue, M x 1024 x 1024) and a store-only GEMM of the same shape
back to back, timing each launch with a HIP event pair; run it bare and under
`rocprofv3 --kernel-trace` and compare the printed event averages with the trace's averages.

  python tools/prof_inflation.py [--iters 50] [--M 65536]
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
from ured_hip import kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--M", type=int, default=65536)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    M, N, Kd = a.M, 1024, 1024
    g = torch.Generator(device=dev).manual_seed(0)
    A = torch.randn(M, Kd, device=dev, generator=g)
    W = torch.randn(Kd, N, device=dev, generator=g) * 0.03
    Y = torch.randn(M, N, device=dev, generator=g)
    C = torch.empty(M, N, device=dev)
    st = K.BNState(torch.zeros(N, device=dev), torch.ones(N, device=dev), torch.ones(N, device=dev),
                   torch.zeros(N, device=dev))
    bws = torch.empty(K.nblocks(M), 2, N, device=dev)
    out = {}
    for name, kw in (("dgrad_bnbwd", dict(b_kmajor=True, epi=K.EPI_BNBWD, Yp=Y, ldy=N, bn=st, bwd_res=False, bwd_ws=bws)),
                     ("store", dict(b_kmajor=True))):
        for _ in range(5):
            K.gemm(M, N, Kd, A, Kd, W, N, C, N, **kw)
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.iters)]
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for e0, e1 in ev:
            e0.record()
            K.gemm(M, N, Kd, A, Kd, W, N, C, N, **kw)
            e1.record()
        t1.record()
        torch.cuda.synchronize()
        per = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
        out[name] = {"event_avg_us": round(1e3 * sum(per) / len(per), 2), "event_median_us": round(1e3 * per[len(per) // 2], 2),
                     "loop_avg_us": round(1e3 * t0.elapsed_time(t1) / a.iters, 2),
                     "tflops_event": round(2.0 * M * N * Kd / (sum(per) / len(per) * 1e-3) / 1e12, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
