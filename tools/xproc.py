"""Cross-process interference probe: one process recomputes the same small-kernel results over and
over (the xyz-edge weight gradient, ured_wgrad_skinny, and a column sum) on fixed inputs and counts
results that differ from the first, while other processes keep the GPU busy with GEMMs.

  python tools/xproc.py check --seconds 20      # the checker
  python tools/xproc.py load --seconds 25       # a GEMM load process (K.gemm dgrad + wgrad shapes)
"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

ge.add_pkg_path()
from ured_hip import kernels as K  # noqa: E402


def check(seconds, interleave=False):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(1)
    M = 32768
    dY = torch.randn(M, 64, device=dev, generator=g)
    x = torch.randn(M, 3, device=dev, generator=g)
    cs_in = torch.randn(M, 512, device=dev, generator=g)

    names = ["skinny wgrad", "colsum", "torch elementwise", "torch row sum", "torch mm"]

    def once():
        dW = torch.empty(64, 3, device=dev)
        K.wgrad(dY, 64, x, 3, 64, 3, M, dW, 3)
        return (dW, K.colsum(cs_in), dY * 1.5 + 0.25, dY.sum(dim=0), dY[:4096].t() @ cs_in[:4096])
    ref = [t.clone() for t in once()]
    torch.cuda.synchronize()
    gemm = _load_setup(dev) if interleave else None
    n = 0
    bad = [0] * len(names)
    t0 = time.time()
    while time.time() - t0 < seconds:
        if gemm is not None:       # a GEMM of this process right before, same stream
            gemm()
            torch.cuda.synchronize()
        out = once()
        torch.cuda.synchronize()
        n += 1
        for i, (o, r) in enumerate(zip(out, ref)):
            bad[i] += not torch.equal(o, r)
    print(f"check: {n} recomputes; differing: " + ", ".join(f"{nm} {b}" for nm, b in zip(names, bad)), flush=True)


def _load_setup(dev):
    g = torch.Generator(device=dev).manual_seed(2)
    M, N, Kd = 62464, 1024, 1024
    dY = torch.randn(M, N, device=dev, generator=g)
    W = torch.randn(N, Kd, device=dev, generator=g) * 0.05
    Y = torch.randn(M, Kd, device=dev, generator=g)
    G = torch.empty(M, Kd, device=dev)
    bws = torch.empty(K.nblocks(M), 2, Kd, device=dev)
    s = torch.rand(Kd, device=dev, generator=g) + 0.5
    t = torch.randn(Kd, device=dev, generator=g) * 0.1
    st = K.BNState(torch.zeros(Kd, device=dev), torch.ones(Kd, device=dev), s, t)
    dW = torch.empty(N, Kd, device=dev)

    def run():
        K.gemm(M, Kd, N, dY, N, W, Kd, G, Kd, b_kmajor=True, epi=K.EPI_BNBWD, Yp=Y, ldy=Kd, bn=st,
               bwd_res=False, bwd_ws=bws)
        K.wgrad(dY, N, Y, Kd, N, Kd, M, dW, Kd, pro=K.PRO_ENC, pro_s=s, pro_t=t)
    return run


def load(seconds):
    run = _load_setup(torch.device("cuda:0"))
    t0 = time.time()
    n = 0
    while time.time() - t0 < seconds:
        for _ in range(10):
            run()
        torch.cuda.synchronize()
        n += 10
    print(f"load: {n} iterations", flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["check", "load"])
    ap.add_argument("--seconds", type=float, default=20)
    ap.add_argument("--interleave", action="store_true", help="check: run a GEMM of this process before each check")
    a = ap.parse_args()
    if a.mode == "check":
        check(a.seconds, a.interleave)
    else:
        load(a.seconds)
