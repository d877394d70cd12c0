"""K / M sweep of the plain-store GEMM (fixed per-block cost vs main-loop rate)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import __graft_entry__ as ge  # noqa: E402
ge.add_pkg_path()
from ured_hip import kernels as K  # noqa: E402
from gemm_bench import timeit  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    for M, N, Ks in ((262144, 1024, (128, 256, 512, 1024, 2048, 4096)), (65536, 1024, (1024,)), (16384, 1024, (1024,)),
                     (262144, 512, (1024,)), (262144, 256, (1024,)), (262144, 128, (1024,))):
        for Kd in Ks:
            X = torch.randn(M, Kd, device=dev, generator=g)
            W = torch.randn(N, Kd, device=dev, generator=g) * 0.05
            Y = torch.empty(M, N, device=dev)
            t = timeit(lambda: K.gemm(M, N, Kd, X, Kd, W, Kd, Y, N), 10)
            blocks = (M // 128) * (N // 128)
            print(f"M={M} N={N} K={Kd}: {t * 1e6:9.1f} us  {2.0 * M * N * Kd / t / 1e12:6.1f} TF  "
                  f"{t * 1e6 / (blocks / 512):7.2f} us/round(512 blocks)", flush=True)
            del X, W, Y


if __name__ == "__main__":
    main()
