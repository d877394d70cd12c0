import sys, copy
sys.path.insert(0, "/root/repo"); import __graft_entry__ as ge; ge.add_pkg_path()
import torch
from attention_graph.attention_gnn import ResidualAttentionMessagePropagation as RAMP
dev = torch.device("cuda:0")
def err(a, b): return (a.detach().double().cpu() - b.detach().double().cpu()).abs().max().item()
C = 512
torch.manual_seed(0)
m = RAMP(C, 4).to(dev).train()
r64 = copy.deepcopy(m).double().cpu()
x0 = torch.randn(16, 2, C, device=dev); x1 = torch.randn(16, 16, C, device=dev)
for mode in ("self_pair", "cross", "single"):
    a0, a1 = x0.clone().requires_grad_(True), x1.clone().requires_grad_(True)
    b0, b1 = x0.double().cpu().requires_grad_(True), x1.double().cpu().requires_grad_(True)
    if mode == "self_pair":
        o0, o1 = m.forward_nodes_self_pair(a0, a1)
        p0 = r64(b0.transpose(1, 2), b0.transpose(1, 2)).transpose(1, 2)
        p1 = r64(b1.transpose(1, 2), b1.transpose(1, 2)).transpose(1, 2)
    elif mode == "cross":
        o0 = m.forward_nodes(a0, a1); o1 = m.forward_nodes(a1, o0)
        p0 = r64(b0.transpose(1, 2), b1.transpose(1, 2)).transpose(1, 2)
        p1 = r64(b1.transpose(1, 2), p0.transpose(1, 2)).transpose(1, 2)
    else:
        o0 = m.forward_nodes(a0); o1 = m.forward_nodes(a1)
        p0 = r64(b0.transpose(1, 2), b0.transpose(1, 2)).transpose(1, 2)
        p1 = r64(b1.transpose(1, 2), b1.transpose(1, 2)).transpose(1, 2)
    g0, g1 = torch.randn_like(o0), torch.randn_like(o1)
    ((o0 * g0).sum() + (o1 * g1).sum()).backward()
    ((p0 * g0.double().cpu()).sum() + (p1 * g1.double().cpu()).sum()).backward()
    print(mode, "out", err(o0, p0), err(o1, p1), "gx0", err(a0.grad, b0.grad), b0.grad.abs().max().item(),
          "gx1", err(a1.grad, b1.grad), b1.grad.abs().max().item())
    rp = dict(r64.named_parameters())
    for k, p in m.named_parameters():
        e = err(p.grad, rp[k].grad); mx = rp[k].grad.abs().max().item()
        if e > 1e-4 * mx: print("   ", k, e, mx)
        p.grad = None; rp[k].grad = None
