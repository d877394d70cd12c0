"""Per-launch GPU time of single node-GEMM launches (csrc/node.hip) at DeformNet shapes: 50 launches
captured in a HIP graph and replayed, so host launch cost is excluded.

  python tools/node_bench.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

ge.add_pkg_path()


def main():
    from ured_hip import node
    dev = torch.device("cuda:0")
    for (M, N, K) in [(32, 512, 32), (32, 512, 512), (32, 1024, 1024), (288, 512, 512), (288, 1536, 512),
                      (256, 1024, 1024), (288, 1024, 1024), (288, 512, 1024), (1024, 1024, 288), (16, 256, 1024),
                      (256, 256, 512)]:
        x = torch.randn(M, K, device=dev)
        W = torch.randn(N, K, device=dev)
        y = torch.empty(M, N, device=dev)
        node.linear(x, W, y)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for _ in range(50):
                    node.linear(x, W, y)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 250
        print(f"G{M}x{N}x{K}: {us:6.2f} us/launch  {2 * M * N * K / us / 1e6:7.2f} TF/s", flush=True)


if __name__ == "__main__":
    main()
