"""Diagnose graph-vs-eager divergence: which gradients / parameters differ after replays."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import __graft_entry__ as ge  # noqa: E402
ge.add_pkg_path()
import torch  # noqa: E402


def main():
    from test_graph_gpu import _make
    from test_dp_gpu import CFG
    from dataset import synthetic
    from engine.graph import GraphedStep
    from engine.train import batch_to_device
    dev = torch.device("cuda:0")
    cfg = dict(CFG, cuda_graph=True)
    batches = [batch_to_device(synthetic.make_batch(2, 128, 24, parts=[3, 2], seed=50 + i), dev) for i in range(4)]
    a, b = _make(dev, cfg), _make(dev, cfg)
    g = GraphedStep(a)
    for i in range(4):
        la = g.step(batches[i])["all_loss"].clone()
        lb = b.step(batches[i])["all_loss"]
        torch.cuda.synchronize()
        print("step", i, "loss equal", torch.equal(la, lb), la.item(), lb.item())
        ngd, npd = 0, 0
        for name in a.models:
            pa = dict(a.models[name].named_parameters())
            for k, p in b.models[name].named_parameters():
                q = pa[k]
                if (p.grad is None) != (q.grad is None):
                    print("  grad presence differs", name, k)
                    continue
                if p.grad is not None and not torch.equal(p.grad, q.grad):
                    ngd += 1
                    if ngd <= 8:
                        print("  grad differs", name, k, (p.grad - q.grad).abs().max().item(), p.grad.abs().max().item())
                if not torch.equal(p, q):
                    npd += 1
                    if npd <= 8:
                        print("  param differs", name, k, (p - q).abs().max().item())
        print("  #grad diffs", ngd, "#param diffs", npd)


if __name__ == "__main__":
    main()
