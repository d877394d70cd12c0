"""Graph-node kernels of csrc/node.hip (DeformNet_MatchingNet's Conv1d / BatchNorm1d layers) vs
float64 torch restatements of the reference layers (attention_graph/attention_gnn.py:8-55,
attention_utils.py:62-86, network/deformation_net.py:61,90).

Tolerances: GEMMs within 1e-5 of the result's largest magnitude (fp32 MFMA, K <= 1536); BN
statistics/activations within 1e-5 relative (fp64 sums); every gradient within 2e-5 relative of
its largest element.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _close(a, b, rtol=1e-5):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    err = (a - b).abs().max().item()
    assert err <= rtol * b.abs().max().item() + 1e-9, err


@pytest.mark.parametrize("M,N,K", [(288, 1536, 512), (32, 1024, 1024), (256, 512, 1024), (7, 6, 256),
                                   (33, 70, 45), (1, 3, 4)])
def test_node_linear_dgrad_wgrad(dev, M, N, K):
    from ured_hip import node
    g = torch.Generator().manual_seed(M * 7 + N + K)
    x = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    R = torch.randn(M, N, generator=g)
    go = torch.randn(M, N, generator=g)
    xd, Wd, bd, Rd = (t.to(dev).requires_grad_(True) for t in (x, W, b, R))
    y = node.node_linear(xd, Wd, bd, Rd)
    y.backward(go.to(dev))
    x64, W64, b64, R64 = (t.double().requires_grad_(True) for t in (x, W, b, R))
    y64 = x64 @ W64.t() + b64 + R64
    y64.backward(go.double())
    _close(y, y64)
    for a, r in ((xd, x64), (Wd, W64), (bd, b64), (Rd, R64)):
        _close(a.grad, r.grad, 2e-5)


def test_node_gemm_epilogue_options(dev):
    """Two A sources split along K (the FFN's cat([x, message])), per-row-group bias, ReLU,
    gate, residual and accumulation, on column-slice views (row strides != widths)."""
    from ured_hip import node
    g = torch.Generator().manual_seed(3)
    M, C, N, P = 64, 128, 96, 16
    big = torch.randn(M, 3 * C, generator=g).to(dev)
    x, msg = big[:, :C], big[:, 2 * C:]
    W = (torch.randn(N, 2 * C, generator=g) / 16).to(dev)
    b = torch.randn(N, generator=g).to(dev)
    rb = torch.randn(M // P, N, generator=g).to(dev)
    gate = torch.randn(M, N, generator=g).to(dev)
    R = torch.randn(M, N, generator=g).to(dev)
    C0 = torch.randn(M, N, generator=g).to(dev)
    out = C0.clone()
    node.node_gemm(M, N, 2 * C, x.data_ptr(), x.stride(0), 1, W.data_ptr(), 1, W.stride(0), out, N,
                   A2=msg.data_ptr(), sam2=msg.stride(0), sak2=1, k1=C, bias=b, rowbias=rb, ldrb=N, rdiv=P,
                   relu_out=True, gate=gate, ldgate=N, R=R, ldR=N, accumulate=True)
    xx = torch.cat([x, msg], 1).double()
    v = xx @ W.double().t() + b.double() + rb.double().repeat_interleave(P, 0)
    v = torch.where(gate.double() > 0, v.clamp(min=0), torch.zeros_like(v)) + R.double() + C0.double()
    _close(out, v)


@pytest.mark.parametrize("off", [(0, 32, 288), (0, 256), (0, 32)])
@pytest.mark.parametrize("training", [True, False])
def test_node_bn_matches_batchnorm1d(dev, off, training):
    """BatchNorm1d after a ReLU per node set (one module call per set, in order): activations,
    running statistics, num_batches_tracked, and the backward (dY through the ReLU, dgamma,
    dbeta) vs torch float64 calls of the module on each set."""
    from ured_hip import node
    g = torch.Generator().manual_seed(len(off) + int(training))
    R, N = off[-1], 1024
    Y = torch.randn(R, N, generator=g)
    G = torch.randn(R, N, generator=g)
    bnm = torch.nn.BatchNorm1d(N).to(dev)
    with torch.no_grad():
        bnm.weight.uniform_(0.5, 1.5)
        bnm.bias.uniform_(-0.2, 0.2)
        bnm.running_mean.uniform_(-0.1, 0.1)
        bnm.running_var.uniform_(0.8, 1.2)
    ref = torch.nn.BatchNorm1d(N).double()
    ref.load_state_dict({k: v.double() if v.dtype.is_floating_point else v for k, v in bnm.state_dict().items()})
    bnm.train(training)
    ref.train(training)
    Yd = Y.to(dev)
    act, mean, invstd = node.bn_fwd(Yd, bnm, off, training)
    Y64 = Y.double().requires_grad_(True)
    outs = [ref(torch.relu(Y64[a:b])) for a, b in zip(off[:-1], off[1:])]
    act64 = torch.cat(outs)
    _close(act, act64)
    _close(bnm.running_mean, ref.running_mean)
    _close(bnm.running_var, ref.running_var)
    assert int(bnm.num_batches_tracked) == int(ref.num_batches_tracked)
    act64.backward(G.double())
    dY, dgamma, dbeta = node.bn_bwd(G.to(dev), Yd, bnm.weight, mean, invstd, off, training)
    _close(dY, Y64.grad, 2e-5)
    _close(dgamma, ref.weight.grad, 2e-5)
    _close(dbeta, ref.bias.grad, 2e-5)


def test_param_decoder_matches_reference(dev):
    """param_decoder (Conv 3C->256 -> ReLU -> Conv 256->6) on cat([g0|g1 broadcast, parts])
    (deformation_net.py:87-91) with the global half as a row bias, forward and backward."""
    from ured_hip import node
    from attention_graph.attention_utils import FeedForwardNet_norm
    torch.manual_seed(0)
    B, P, C = 16, 16, 512
    dec = FeedForwardNet_norm([3 * C, 256, 6], use_norm="None").to(dev)
    ref = FeedForwardNet_norm([3 * C, 256, 6], use_norm="None").double()
    ref.load_state_dict({k: v.double() for k, v in dec.state_dict().items()})
    glob = torch.randn(B, 2 * C, device=dev, requires_grad=True)
    parts = torch.randn(B * P, C, device=dev, requires_grad=True)
    out = node.param_decoder(dec, glob, parts, P)
    go = torch.randn_like(out)
    out.backward(go)
    g64, p64 = glob.detach().double().cpu().requires_grad_(True), parts.detach().double().cpu().requires_grad_(True)
    full = torch.cat([g64.repeat_interleave(P, 0), p64], 1)                      # [B*P, 3C]
    h = torch.relu(full @ ref[0].weight.view(256, -1).t() + ref[0].bias)
    r = h @ ref[2].weight.view(6, -1).t() + ref[2].bias
    r.backward(go.double().cpu())
    _close(out, r)
    _close(glob.grad, g64.grad, 2e-5)
    _close(parts.grad, p64.grad, 2e-5)
    for k in ("0.weight", "0.bias", "2.weight", "2.bias"):
        _close(dict(dec.named_parameters())[k].grad, dict(ref.named_parameters())[k].grad, 2e-5)


def test_batched_jobs_equal_single_launches(dev):
    """Up to four independent GEMMs of different shapes and operand layouts in one launch give
    exactly (bitwise) the results of separate launches."""
    from ured_hip import node
    g = torch.Generator().manual_seed(9)
    mk = lambda *s: torch.randn(*s, generator=g).to(dev)   # noqa: E731
    x1, W1 = mk(32, 512), mk(512, 512)
    x2, W2 = mk(256, 512), mk(1024, 512)
    gr, Wd = mk(288, 1536), mk(1536, 512)
    gw, xw = mk(288, 1024), mk(288, 200)
    outs_b = [torch.empty(32, 512, device=dev), torch.empty(256, 1024, device=dev), torch.empty(288, 512, device=dev),
              torch.empty(1024, 200, device=dev)]
    outs_s = [torch.empty_like(o) for o in outs_b]
    mkd = lambda o: [node.linear_desc(x1, W1, o[0]), node.linear_desc(x2, W2, o[1]),   # noqa: E731
                     node.dgrad_desc(gr, Wd, o[2]), node.wgrad_desc(gw, xw, o[3])]
    node.launch(*mkd(outs_b))
    for d in mkd(outs_s):
        node.launch(d)
    for a, b in zip(outs_b, outs_s):
        assert torch.equal(a, b)
    _close(outs_b[2], gr.double() @ Wd.double())
    _close(outs_b[3], gw.double().t() @ xw.double())


def test_v4_equals_v1_bitwise(dev):
    """csrc/node.hip runs a launch on the v4 kernel (two half-chunks in flight, buffer loads) when
    every job has K, k1, n1 multiples of 32, else on v1. A job with K = 45 in the batch forces v1
    for all of them; the same jobs launched one by one take v4: same chunk -> wave assignment, MFMA
    order and combine, so bitwise the same, for every operand-layout combination (k-contiguous /
    strided A and B), a split A (k1 = 64) and accumulation."""
    from ured_hip import node
    g = torch.Generator().manual_seed(11)
    mk = lambda *s: torch.randn(*s, generator=g).to(dev)   # noqa: E731
    x, W = mk(288, 1536), mk(512, 1536)          # A, B k-contiguous (forward)
    gr, Wd = mk(288, 1024), mk(1024, 512)        # A k-contiguous, B strided (dgrad)
    gw, xw = mk(288, 256), mk(288, 96)           # A, B strided (wgrad)
    xs, ms, Ws = mk(64, 64), mk(64, 96), mk(128, 160)   # split A (k1 = 64)
    xo, Wo = mk(40, 45), mk(20, 45)              # K = 45: v1 only
    c0 = mk(256, 96)                             # accumulated into by the wgrad job

    def jobs(o):
        o[3].copy_(c0)
        return [node.linear_desc(x, W, o[0]), node.dgrad_desc(gr, Wd, o[1]),
                node.node_gemm_desc(64, 128, 160, xs.data_ptr(), xs.stride(0), 1, Ws.data_ptr(), 1, Ws.stride(0),
                                    o[2], 128, A2=ms.data_ptr(), sam2=ms.stride(0), sak2=1, k1=64),
                node.wgrad_desc(gw, xw, o[3], accumulate=True),
                node.linear_desc(xo, Wo, o[4])]

    shapes = [(288, 512), (288, 512), (64, 128), (256, 96), (40, 20)]
    ob = [torch.empty(*s, device=dev) for s in shapes]
    os_ = [torch.empty(*s, device=dev) for s in shapes]
    node.launch(*jobs(ob))                       # v1 (the K = 45 job)
    for d in jobs(os_):
        node.launch(d)                           # v4 for all but the last
    for i in range(5):
        assert torch.equal(ob[i], os_[i]), i
    _close(ob[0], x.double() @ W.double().t())
    _close(ob[1], gr.double() @ Wd.double())
    _close(ob[2], torch.cat([xs, ms], 1).double() @ Ws.double().t())
    _close(ob[3], gw.double().t() @ xw.double() + c0.double())


@pytest.mark.parametrize("sets", [(0, 32, 288), (0, 32)])
def test_node_ffn_and_linear2_match_reference(dev, sets):
    """ResidualAttentionMessagePropagation's FFN update out = x + conv2(BN(relu(conv1(cat([x, m])))))
    per node set, and the paired q / k|v projections, forward and backward vs float64."""
    from ured_hip import node
    from attention_graph.attention_utils import FeedForwardNet_norm
    torch.manual_seed(1)
    C = 512
    R = sets[-1]
    fc = FeedForwardNet_norm([2 * C, 2 * C, C], use_norm="use_bn").to(dev).train()
    ref = FeedForwardNet_norm([2 * C, 2 * C, C], use_norm="use_bn").double().train()
    ref.load_state_dict({k: v.double() if v.dtype.is_floating_point else v for k, v in fc.state_dict().items()})
    x = torch.randn(R, C, device=dev, requires_grad=True)
    m = torch.randn(R, C, device=dev, requires_grad=True)
    out = node.node_ffn(fc, x, m, None, sets)
    go = torch.randn_like(out)
    out.backward(go)
    x64, m64 = x.detach().double().cpu().requires_grad_(True), m.detach().double().cpu().requires_grad_(True)
    h = torch.cat([x64, m64], 1)
    y = h @ ref[0].weight.view(2 * C, -1).t() + ref[0].bias
    parts = [ref[2](torch.relu(y[a:b])) for a, b in zip(sets[:-1], sets[1:])]
    r = x64 + torch.cat(parts) @ ref[3].weight.view(C, -1).t() + ref[3].bias
    r.backward(go.double().cpu())
    _close(out, r)
    _close(x.grad, x64.grad, 2e-5)
    _close(m.grad, m64.grad, 2e-5)
    rp = dict(ref.named_parameters())
    for k, p in fc.named_parameters():
        _close(p.grad, rp[k].grad, 2e-5)
    _close(fc[2].running_mean, ref[2].running_mean)
    _close(fc[2].running_var, ref[2].running_var)
    # paired projections
    xq = torch.randn(32, C, device=dev, requires_grad=True)
    xk = torch.randn(256, C, device=dev, requires_grad=True)
    Wq, bq = torch.randn(C, C, device=dev, requires_grad=True), torch.randn(C, device=dev, requires_grad=True)
    # k and v weights / biases: adjacent slices of one buffer (the FlatAdam layout, read as one
    # matrix) or separate tensors (concatenated inside the Function)
    for adjacent in (True, False):
        if adjacent:
            wbuf, bbuf = torch.randn(2 * C * C, device=dev), torch.randn(2 * C, device=dev)
            Wk1, Wk2 = (wbuf[i * C * C:(i + 1) * C * C].view(C, C).detach().requires_grad_(True) for i in (0, 1))
            bk1, bk2 = (bbuf[i * C:(i + 1) * C].detach().requires_grad_(True) for i in (0, 1))
            assert node.fused_rows([Wk1, Wk2]) is not None
        else:
            Wk1, Wk2 = (torch.randn(C, C, device=dev, requires_grad=True) for _ in (0, 1))
            bk1, bk2 = (torch.randn(C, device=dev, requires_grad=True) for _ in (0, 1))
            assert node.fused_rows([Wk1, Wk2]) is None
        for t in (xq, xk, Wq, bq):
            t.grad = None
        q, kv = node.node_proj((xq, xk), [(Wq,), (Wk1, Wk2)], [(bq,), (bk1, bk2)])
        gq, gk = torch.randn_like(q), torch.randn_like(kv)
        (q * gq).sum().backward(retain_graph=True)
        (kv * gk).sum().backward()
        leaves = (xq, Wq, bq, xk, Wk1, Wk2, bk1, bk2)
        ts = [t.detach().double().cpu().requires_grad_(True) for t in leaves]
        q64 = ts[0] @ ts[1].t() + ts[2]
        k64 = ts[3] @ torch.cat([ts[4], ts[5]]).t() + torch.cat([ts[6], ts[7]])
        ((q64 * gq.double().cpu()).sum() + (k64 * gk.double().cpu()).sum()).backward()
        _close(q, q64)
        _close(kv, k64)
        for a, b in zip(leaves, ts):
            _close(a.grad, b.grad, 2e-5)
