"""Micro-benchmark of ured_gemm on the U-RED step's dominant layer shapes (config 2).

  python tools/gemm_bench.py [--iters 20] [--step] [--lib]
Prints TFLOP/s per (shape, variant); interleaves variants in one process (rule 24).
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

SHAPES = [  # (name, M, N, K)  — source encoder (M = 16*16*1024 points)
    ("src.fuse 1024->1024", 262144, 1024, 1024),
    ("src.ppo0 1024->512", 262144, 512, 1024),
    ("src.ppo3 512->512", 262144, 512, 512),
    ("src.mlp2.6 128->1024", 262144, 1024, 128),
    ("recon_src R1 512->256", 262144, 256, 512),
]
STEP_SHAPES = [  # config-2 step sizes (unique-source encoding: M = 32768 target points, ~62-64 k source points)
    ("step src.fuse 1024->1024", 62464, 1024, 1024),
    ("step src.ppo0 1024->512", 62464, 512, 1024),
    ("step tgt.ppo3 512->512", 32768, 512, 512),
    ("step tgt.mlp 128->1024", 32768, 1024, 128),
    ("step R1 512->256", 32768, 256, 512),
    ("step R3 256->32", 32768, 32, 256),
]


def timeit(fn, iters):
    for _ in range(3):
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
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--step", action="store_true", help="the config-2 step's layer sizes instead of M=262144")
    ap.add_argument("--lib", action="store_true",
                    help="also time torch.mm (the ROCm BLAS library, fp32) on the same plain products")
    ap.add_argument("--dgrad-layouts", action="store_true",
                    help="also time store-only dgrad with the weight k-major vs pre-transposed (row-major)")
    a = ap.parse_args()
    ge.build()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    out = {}
    for name, M, N, Kd in (STEP_SHAPES if a.step else SHAPES):
        X = torch.randn(M, Kd, device=dev, generator=g)
        W = torch.randn(N, Kd, device=dev, generator=g) * 0.05
        s = torch.rand(Kd, device=dev, generator=g) + 0.5
        t = torch.randn(Kd, device=dev, generator=g) * 0.1
        Y = torch.empty(M, N, device=dev)
        ws = torch.empty(K.nblocks(M), 2, N, device=dev)
        dY = torch.randn(M, N, device=dev, generator=g)
        G = torch.empty(M, Kd, device=dev)
        bws = torch.empty(K.nblocks(M), 2, Kd, device=dev)
        st = K.BNState(torch.zeros(Kd, device=dev), torch.ones(Kd, device=dev), s, t)
        dW = torch.empty(N, Kd, device=dev)
        t2 = torch.rand(N, device=dev, generator=g) + 0.5      # prologue scale / shift over the dgrad's K = N
        flop = 2.0 * M * N * Kd
        r = {}
        r["fwd"] = flop / timeit(lambda: K.gemm(M, N, Kd, X, Kd, W, Kd, Y, N, pro_a=K.PRO_ENC, pro_s=s, pro_t=t,
                                                epi=K.EPI_FWD, stat_ws=ws), a.iters) / 1e12
        r["fwd_store"] = flop / timeit(lambda: K.gemm(M, N, Kd, X, Kd, W, Kd, Y, N), a.iters) / 1e12
        r["pro_store"] = flop / timeit(lambda: K.gemm(M, N, Kd, X, Kd, W, Kd, Y, N, pro_a=K.PRO_ENC, pro_s=s,
                                                      pro_t=t), a.iters) / 1e12
        r["stats_nopro"] = flop / timeit(lambda: K.gemm(M, N, Kd, X, Kd, W, Kd, Y, N, epi=K.EPI_FWD, stat_ws=ws),
                                         a.iters) / 1e12
        r["dgrad_bnbwd"] = flop / timeit(lambda: K.gemm(M, Kd, N, dY, N, W, Kd, G, Kd, b_kmajor=True, epi=K.EPI_BNBWD,
                                                        Yp=X, ldy=Kd, bn=st, bwd_ws=bws), a.iters) / 1e12
        try:   # measurement build only (-DURED_EXP_DGRAD_PRO=1): the dgrad with a one-input A prologue
            r["dgrad_bnbwd_pro"] = flop / timeit(lambda: K.gemm(M, Kd, N, dY, N, W, Kd, G, Kd, b_kmajor=True,
                                                                epi=K.EPI_BNBWD, Yp=X, ldy=Kd, bn=st, bwd_ws=bws,
                                                                pro_a=K.PRO_ENC, pro_s=t2, pro_t=t2), a.iters) / 1e12
        except Exception:
            pass
        if a.dgrad_layouts:
            Wt = W.t().contiguous()   # [Kd][N]: the dgrad B operand row-major (k = N contiguous)
            r["dgrad_store"] = flop / timeit(lambda: K.gemm(M, Kd, N, dY, N, W, Kd, G, Kd, b_kmajor=True), a.iters) / 1e12
            r["dgrad_store_T"] = flop / timeit(lambda: K.gemm(M, Kd, N, dY, N, Wt, N, G, Kd), a.iters) / 1e12
        r["wgrad"] = flop / timeit(lambda: K.wgrad(dY, N, X, Kd, N, Kd, M, dW, Kd, pro=K.PRO_ENC, pro_s=s, pro_t=t),
                                   a.iters) / 1e12
        if a.lib:
            torch.backends.cuda.matmul.allow_tf32 = False
            Yl = torch.empty(M, N, device=dev)
            Gl = torch.empty(M, Kd, device=dev)
            dWl = torch.empty(N, Kd, device=dev)
            r["lib_fwd"] = flop / timeit(lambda: torch.mm(X, W.t(), out=Yl), a.iters) / 1e12
            r["lib_dgrad"] = flop / timeit(lambda: torch.mm(dY, W, out=Gl), a.iters) / 1e12
            r["lib_wgrad"] = flop / timeit(lambda: torch.mm(dY.t(), X, out=dWl), a.iters) / 1e12
            del Yl, Gl, dWl
        out[name] = {k: round(v, 1) for k, v in r.items()}
        print(name, out[name], flush=True)
        del X, W, Y, ws, dY, G, bws, dW
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
