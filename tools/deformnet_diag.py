"""DeformNet node-major path vs the channel-first fp32 / float64 runs (tests/test_attn_gpu.py's
comparison), printing every deviating gradient; bisection variants via argv:
  seq     node GEMM jobs launched one per launch (no batching)
  nolin2  cross-attention q and k|v projections as two NodeLinearFn calls
  noffn   FeedForwardNet_norm update on torch ops (F.linear + BatchNorm1d)
  nopd    param_decoder on torch ops
"""
import copy
import os
import sys

sys.path.insert(0, "/root/repo")
import __graft_entry__ as ge  # noqa: E402
ge.add_pkg_path()
import torch  # noqa: E402
sys.path.insert(0, "/root/repo/tests")
from test_attn_gpu import _channel_first_forward, _err  # noqa: E402
from network.deformation_net import DeformNet_MatchingNet  # noqa: E402
from ured_hip import node  # noqa: E402
import attention_graph.attention_gnn as agn  # noqa: E402

if "seq" in sys.argv:
    orig = node.launch
    node.launch = lambda *ds: [orig(d) for d in ds]
if "noproj" in sys.argv:    # each projection group as its own launch
    def _split_proj(xs, ws, bs, aliases=None):
        al = tuple(aliases) if aliases is not None else (False,) * len(xs)
        if len(xs) == 1:
            return node.node_proj(xs, ws, bs, aliases=al)
        outs = [node.node_proj((x,), [w], [b], aliases=(a,)) for x, w, b, a in zip(xs, ws, bs, al)]
        ys = [o[0] if a else o for o, a in zip(outs, al)]
        return tuple(ys) + tuple(o[1] for o, a in zip(outs, al) if a)
    agn.node_proj = _split_proj
if "noffn" in sys.argv:
    agn.ResidualAttentionMessagePropagation._node_ffn_ok = lambda self: False
if "nopd" in sys.argv:
    import network.deformation_net as dnm
    dnm.node_param_decoder = lambda dec, glob, parts, P: dec.forward_nodes(
        torch.cat([glob.repeat_interleave(P, 0), parts], -1).unsqueeze(0))[0]
dev = torch.device("cuda:0")
for C in [int(a) for a in sys.argv[1:] if a.isdigit()] or (512,):
    torch.manual_seed(C + int(os.environ.get('SEED', '0')))
    net = DeformNet_MatchingNet(3 * C, graph_dim=C, max_num_parts=16, matching=False).to(dev).train()
    ref = copy.deepcopy(net)
    ref64 = copy.deepcopy(net).double()
    tf = torch.randn(16, C, device=dev)
    sp = torch.randn(16, 16, C, device=dev)
    a_t, a_s = tf.clone().requires_grad_(True), sp.clone().requires_grad_(True)
    b_t, b_s = tf.clone().requires_grad_(True), sp.clone().requires_grad_(True)
    c_t, c_s = tf.double().requires_grad_(True), sp.double().requires_grad_(True)
    out = net(a_t, a_s, None)
    rout = _channel_first_forward(ref, b_t, b_s)
    tout = _channel_first_forward(ref64, c_t, c_s)
    go = torch.randn_like(out)
    out.backward(go)
    rout.backward(go)
    tout.backward(go.double())
    print(sys.argv[1:], "C", C, "out", _err(out, tout), _err(rout, tout), "tf", _err(a_t.grad, c_t.grad),
          _err(b_t.grad, c_t.grad), "sp", _err(a_s.grad, c_s.grad), _err(b_s.grad, c_s.grad))
    def nerr(a, b):
        a, b = a.detach().double().cpu(), b.detach().double().cpu()
        return ((a - b).norm() / b.norm().clamp(min=1e-30)).item()
    rp_, tp_ = dict(ref.named_parameters()), dict(ref64.named_parameters())
    ratios = []
    for k, p in net.named_parameters():
        if p.grad is None:
            continue
        e1, e2 = nerr(p.grad, tp_[k].grad), nerr(rp_[k].grad, tp_[k].grad)
        ratios.append((e1, e2, k))
    import statistics
    print("  norm-rel errors ours: median %.2e max %.2e | fp32 ref: median %.2e max %.2e" % (
        statistics.median(r[0] for r in ratios), max(r[0] for r in ratios),
        statistics.median(r[1] for r in ratios), max(r[1] for r in ratios)))
    rp, tp = dict(ref.named_parameters()), dict(ref64.named_parameters())
    nbad = 0
    for k, p in net.named_parameters():
        if p.grad is None:
            continue
        e1, e2 = _err(p.grad, tp[k].grad), _err(rp[k].grad, tp[k].grad)
        m = tp[k].grad.abs().max().item()
        if e1 > 3 * e2 + 1e-5 * m:
            nbad += 1
            if nbad <= 6:
                print("  BAD", k, e1, e2, m)
    print("  bad params:", nbad)
