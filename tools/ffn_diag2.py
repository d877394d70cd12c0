import sys, copy
sys.path.insert(0, "/root/repo"); import __graft_entry__ as ge; ge.add_pkg_path()
import torch
from attention_graph.attention_gnn import ResidualAttentionMessagePropagation as RAMP
from ured_hip import node
dev = torch.device("cuda:0")
def err(a, b): return (a.detach().double().cpu() - b.detach().double().cpu()).abs().max().item()
C = 512
torch.manual_seed(0)
m = RAMP(C, 4).to(dev).train()
r64 = copy.deepcopy(m).double().cpu()
r32 = copy.deepcopy(m)
for M, seed in ((256, 1), (32, 2), (288, 3)):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(M, C, generator=g); ms = torch.randn(M, C, generator=g); go = torch.randn(M, C, generator=g)
    for scale in (1.0, 10.0):
        xa, ma = (x * scale).to(dev).requires_grad_(True), ms.to(dev).requires_grad_(True)
        xb, mb = (x * scale).double().requires_grad_(True), ms.double().requires_grad_(True)
        o = node.node_ffn(m.fc, xa, ma, None, (0, M))
        p = xb + r64.fc(torch.cat([xb, mb], 1).t().unsqueeze(0))[0].t()
        xc, mc = (x * scale).to(dev).requires_grad_(True), ms.to(dev).requires_grad_(True)
        q32 = xc + r32.fc(torch.cat([xc, mc], 1).t().unsqueeze(0))[0].t()
        q32.backward(go.to(dev))
        o.backward(go.to(dev)); p.backward(go.double())
        print("   torch fp32: gx", err(xc.grad, xb.grad), "fc.0.weight", err(r32.fc[0].weight.grad, None) if False else "")
        print(M, scale, "out", err(o, p), "gx", err(xa.grad, xb.grad), xb.grad.abs().max().item(), "gm", err(ma.grad, mb.grad))
        rp = dict(r64.fc.named_parameters())
        r3 = dict(r32.fc.named_parameters())
        for k, q in m.fc.named_parameters():
            e = err(q.grad, rp[k].grad); mx = rp[k].grad.abs().max().item()
            e3 = err(r3[k].grad.view_as(rp[k].grad), rp[k].grad)
            if e > 1e-4 * mx or e3 > 1e-4 * mx: print("   ", k, "ours", e, "torch32", e3, mx)
            q.grad = None; rp[k].grad = None; r3[k].grad = None
