"""Per-launch shapes and times of the node GEMM launches of one DeformNet_MatchingNet forward +
backward at the training step's shape (B=16, C=512, 16 part slots): HIP events around every
ured_node_gemm_batch call (synchronous timing, for attribution only).

  python tools/node_shapes.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

ge.add_pkg_path()


def main():
    from network.deformation_net import DeformNet_MatchingNet
    from ured_hip import node
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    C = 512
    net = DeformNet_MatchingNet(3 * C, graph_dim=C, max_num_parts=16, matching=False).to(dev).train()
    tf = torch.randn(16, C, device=dev, requires_grad=True)
    sp = torch.randn(16, 16, C, device=dev, requires_grad=True)
    log = []
    orig = node.launch

    def timed(*descs):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        orig(*descs)
        e1.record()
        log.append((e0, e1, [(d.kind, d.M, d.N, d.K) for d in descs]))

    def once():
        out = net(tf, sp, None)
        out.sum().backward()
    for _ in range(3):
        once()
    torch.cuda.synchronize()
    node.launch = timed
    once()
    torch.cuda.synchronize()
    node.launch = orig
    tot = 0.0
    for e0, e1, jobs in log:
        ms = e0.elapsed_time(e1)
        tot += ms
        fl = sum(2.0 * M * N * K for kind, M, N, K in jobs)
        print(f"{ms * 1e3:7.1f} us {fl / (ms * 1e-3) / 1e12 if ms > 0 else 0:6.2f} TF  " +
              "  ".join(f"{'C' if kind else 'G'}{M}x{N}x{K}" for kind, M, N, K in jobs))
    print(f"{len(log)} launches, {tot * 1e3:.1f} us")


if __name__ == "__main__":
    main()
