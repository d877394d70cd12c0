"""Accuracy of the GEMM path in the loaded libured_hip.so (URED_LIB selects a build) against a
float64 matmul of the same fp32 inputs, at the step's shapes: fwd (row-major A with the BN+ReLU
prologue) and dgrad and wgrad, relative error max |y - y64| / max |y64| and the RMS of
|y - y64| / rms(y64). Run once per build to compare the native fp32 MFMA with the bf16x3 split.

  URED_LIB=build_ab/emu1.so python tools/emu_accuracy.py
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

ge.add_pkg_path()
from ured_hip import kernels as K  # noqa: E402


def err(y, r):
    d = (y.double() - r)
    return {"max_rel": float(d.abs().max() / r.abs().max()), "rms_rel": float(d.pow(2).mean().sqrt() / r.pow(2).mean().sqrt())}


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    out = {}
    for M, N, Kd in [(32768, 1024, 1024), (32768, 512, 512), (62464, 256, 1024), (32768, 1024, 128)]:
        X = torch.randn(M, Kd, device=dev, generator=g)
        W = torch.randn(N, Kd, device=dev, generator=g) * (1.0 / Kd ** 0.5)
        s = torch.rand(Kd, device=dev, generator=g) + 0.5
        t = torch.randn(Kd, device=dev, generator=g) * 0.1
        Y = torch.empty(M, N, device=dev)
        K.gemm(M, N, Kd, X, Kd, W, Kd, Y, N, pro_a=K.PRO_ENC, pro_s=s, pro_t=t)
        A64 = torch.relu(X.double() * s.double() + t.double())
        r = {"fwd": err(Y, A64 @ W.double().t())}
        dY = torch.randn(M, N, device=dev, generator=g)
        G = torch.empty(M, Kd, device=dev)
        K.gemm(M, Kd, N, dY, N, W, Kd, G, Kd, b_kmajor=True)
        r["dgrad"] = err(G, dY.double() @ W.double())
        dW = torch.empty(N, Kd, device=dev)
        K.wgrad(dY, N, X, Kd, N, Kd, M, dW, Kd)
        r["wgrad"] = err(dW, dY.double().t() @ X.double())
        key = f"{M}x{N}x{Kd}"
        out[key] = r
        print(key, json.dumps(r), flush=True)
        del X, W, Y, dY, G, dW, A64
        torch.cuda.empty_cache()
    print(json.dumps({"lib": os.environ.get("URED_LIB", "default"), "errors": out}))


if __name__ == "__main__":
    main()
