"""Parameter gradients written straight into FlatAdam's flat gradient (ured_hip.optim.grad_slot,
the chained q|k|v layout of attention_graph/attention_gnn.py, NodeProjFn) are bit-identical to
autograd's own gradients of the same kernels: first uses write the flat views, the second use of
each cross-attention parameter accumulates in the kernel (call-2 gradient + call-1 gradient, the
order autograd's add uses), the q|k|v weights are read as one matrix without concatenation."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("C", [64, 512])
def test_deformnet_flat_grads_equal_autograd(dev, C):
    from network.deformation_net import DeformNet_MatchingNet
    from ured_hip.node import fused_rows
    from ured_hip.optim import FlatAdam
    torch.manual_seed(C)
    net = DeformNet_MatchingNet(3 * C, graph_dim=C, max_num_parts=16, matching=False).to(dev).train()
    ref = copy.deepcopy(net)                    # plain autograd (deepcopy drops the chain marks)
    params = [p for p in net.parameters() if p.requires_grad]
    opt = FlatAdam(params, [params], lr=0.0)
    tf = torch.randn(16, C, device=dev)
    sp = torch.randn(16, 16, C, device=dev)
    go = torch.randn(16, 16, 6, device=dev)
    net(tf, sp, None).backward(go)              # first step lays out the flat buffers
    opt.step()                                  # lr = 0: parameters unchanged
    mha = net.graph_attention_net.layers[0].module.mha
    ws = [c.weight for c in (mha.in_proj_q, mha.in_proj_k, mha.in_proj_v)]
    assert fused_rows(ws) is not None, "q|k|v weights not laid out back to back"
    opt.zero_grad(set_to_none=True)
    net(tf, sp, None).backward(go)
    opt.gather_grads()
    ref(tf, sp, None).backward(go)
    views = {id(p): v for p, v in zip(opt.params_all, opt._gviews)}
    rp = dict(ref.named_parameters())
    n_inplace = 0
    for k, p in net.named_parameters():
        r = rp[k].grad
        if r is None:
            assert p.grad is None, k
            continue
        assert torch.equal(p.grad, r), (k, (p.grad - r).abs().max().item())
        n_inplace += int(p.grad.data_ptr() == views[id(p)].data_ptr())
    assert n_inplace == sum(1 for p in net.parameters() if p.grad is not None)
