"""GEMM variants at odd shapes / strides against float64 (max |d| / max |ref|), for the HIP build in
use (URED_LIB): a quick bisection aid for tests/test_mlp_gpu.py failures.

  python tools/gemm_cases.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

ge.add_pkg_path()
from ured_hip import kernels as K  # noqa: E402


def rel(y, r):
    return float((y.double() - r).abs().max() / r.abs().max())


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    for M, N, Kd, ldw in [(768, 1024, 1024, 1040), (768, 1024, 1024, 1024), (768, 128, 1024, 1024),
                          (768, 64, 64, 64), (768, 64, 128, 128), (32768, 1024, 1024, 1040)]:
        dY = torch.randn(M, Kd, device=dev, generator=g)
        Wf = torch.randn(Kd, ldw, device=dev, generator=g) * Kd ** -0.5       # [out = K][in >= N]
        G = torch.empty(M, N, device=dev)
        K.gemm(M, N, Kd, dY, Kd, Wf, ldw, G, N, b_kmajor=True)
        e_store = rel(G, dY.double() @ Wf[:, :N].double())
        X = torch.randn(M, N, device=dev, generator=g)
        s = torch.rand(N, device=dev, generator=g) + 0.5
        t = torch.randn(N, device=dev, generator=g) * 0.1
        Y = torch.empty(M, Kd, device=dev)
        K.gemm(M, Kd, N, X, N, Wf[:, :N].contiguous(), N, Y, Kd, pro_a=K.PRO_ENC, pro_s=s, pro_t=t)
        e_fwd = rel(Y, torch.relu(X.double() * s.double() + t.double()) @ Wf[:, :N].double().t())
        dW = torch.empty(Kd, N, device=dev)
        K.wgrad(dY, Kd, X, N, Kd, N, M, dW, N, pro=K.PRO_ENC, pro_s=s, pro_t=t)
        e_wg = rel(dW, dY.double().t() @ torch.relu(X.double() * s.double() + t.double()))
        print(f"M={M:6d} N={N:5d} K={Kd:5d} ldw={ldw:5d}: dgrad(k-major B) {e_store:.2e}  fwd+pro {e_fwd:.2e}  "
              f"wgrad+pro {e_wg:.2e}", flush=True)


if __name__ == "__main__":
    main()
