"""Per-launch GPU time of the node BatchNorm kernels (csrc/node.hip ured_node_bn_fwd / _bwd) at
DeformNet's shapes (288 node rows in two sets of 32 + 256, or one set; N = 1024 / 512): 50 launches
captured in a HIP graph and replayed.

  python tools/node_bn_bench.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

ge.add_pkg_path()


def per_launch_us(fn, n=50):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g):
            for _ in range(n):
                fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / (5 * n)


def main():
    from ured_hip import node
    dev = torch.device("cuda:0")
    for N, off in [(1024, (0, 32, 288)), (1024, (0, 288)), (512, (0, 256))]:
        R = off[-1]
        bnm = torch.nn.BatchNorm1d(N).to(dev).train()
        Y = torch.randn(R, N, device=dev)
        G = torch.randn(R, N, device=dev)
        st = {}

        def fwd():
            st["r"] = node.bn_fwd(Y, bnm, off, True)
        fwd()
        _, mean, invstd = st["r"]
        t_f = per_launch_us(fwd)
        t_b = per_launch_us(lambda: node.bn_bwd(G, Y, bnm.weight, mean, invstd, off, True))
        print(f"N={N} sets={len(off) - 1} rows={R}: fwd {t_f:6.2f} us  bwd {t_b:6.2f} us", flush=True)


if __name__ == "__main__":
    main()
