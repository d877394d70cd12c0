"""DeformNet_MatchingNet forward + backward at the training step's shape (B=16, C=512, 16 part
slots) on its own: ms per call (HIP events), for A/B of the node kernels. --graph: one forward +
backward captured in a HIP graph and replayed (device time, no host launch cost).

  python tools/deformnet_bench.py [--iters 50] [--graph]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

ge.add_pkg_path()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--graph", action="store_true")
    a = ap.parse_args()
    from network.deformation_net import DeformNet_MatchingNet
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    C = 512
    net = DeformNet_MatchingNet(3 * C, graph_dim=C, max_num_parts=16, matching=False).to(dev).train()
    tf = torch.randn(16, C, device=dev, requires_grad=True)
    sp = torch.randn(16, 16, C, device=dev, requires_grad=True)

    def once():
        out = net(tf, sp, None)
        out.sum().backward()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(5):
            once()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    run = once
    if a.graph:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            once()
        run = g.replay
        run()
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        run()
    e1.record()
    torch.cuda.synchronize()
    print(f"deformnet fwd+bwd{' (graph)' if a.graph else ''}: {e0.elapsed_time(e1) / a.iters:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
