"""FlatAdam's flat-gradient claims (ured_hip.optim.grad_slot / grad_buffer, used by the HIP layers'
backward to write parameter gradients straight into the flat buffer), on CPU tensors with a
torch-op autograd Function standing in for a HIP layer:
  * first use of a parameter in a backward: its flat view, adopted by autograd as p.grad (no copy);
  * second use in the same backward: the same view with accumulate=True, the Function adds its
    gradient there and returns None, and p.grad == the sum of both uses (autograd's own value);
  * a gradient kept from an earlier backward (no zero_grad): a fresh tensor, autograd accumulates;
  * no flat layout yet: a fresh tensor;
  * chained parameters (attention q|k|v) laid out back to back, read as one matrix (fused_rows).
"""
import pytest
import torch

from ured_hip.optim import FlatAdam, grad_slot


class _Lin(torch.autograd.Function):
    """y = x W^T with the weight gradient written through grad_slot (as the node layers do)."""

    @staticmethod
    def forward(ctx, x, W):
        ctx.save_for_backward(x, W)
        return x @ W.t()

    @staticmethod
    def backward(ctx, g):
        x, W = ctx.saved_tensors
        buf, acc = grad_slot(W)
        gw = g.t() @ x
        if acc:
            buf.add_(gw)
        else:
            buf.copy_(gw)
        return g @ W, (None if acc else buf)


def _setup():
    torch.manual_seed(0)
    W = torch.nn.Parameter(torch.randn(5, 3))
    V = torch.nn.Parameter(torch.randn(5, 3))
    opt = FlatAdam([W, V], [[W, V]], lr=0.0)
    x = torch.randn(4, 3)
    (_Lin.apply(x, W).sum() + _Lin.apply(x, V).sum()).backward()
    opt.prepare()                                   # lays out the flat buffers (as step() does)
    return W, V, opt, x


def _view(opt, p):
    i = [id(q) for q in opt.params_all].index(id(p))
    return opt._gviews[i]


def test_first_use_writes_the_flat_view():
    W, V, opt, x = _setup()
    opt.zero_grad(set_to_none=True)
    (_Lin.apply(x, W) * 2).sum().backward()
    assert W.grad.data_ptr() == _view(opt, W).data_ptr()
    assert torch.allclose(W.grad, 2 * torch.ones(4, 5).t() @ x)


def test_second_use_accumulates_in_place():
    W, V, opt, x = _setup()
    x2 = torch.randn(4, 3)
    opt.zero_grad(set_to_none=True)
    y = _Lin.apply(x, W)
    (_Lin.apply(y @ torch.randn(5, 3) * 0 + x2, W).sum() + y.sum()).backward()
    assert W.grad.data_ptr() == _view(opt, W).data_ptr()
    ref = torch.ones(4, 5).t() @ x + torch.ones(4, 5).t() @ x2
    assert torch.allclose(W.grad, ref, atol=1e-5)


def test_kept_gradient_accumulates_through_autograd():
    W, V, opt, x = _setup()
    opt.zero_grad(set_to_none=True)
    _Lin.apply(x, W).sum().backward()
    first = W.grad.clone()
    _Lin.apply(x, W).sum().backward()               # no zero_grad: autograd adds a fresh tensor
    assert torch.allclose(W.grad, 2 * first)


def test_no_layout_gives_fresh_tensor():
    W = torch.nn.Parameter(torch.randn(5, 3))
    FlatAdam([W], [[W]], lr=0.0)                     # not flattened until its first step
    buf, acc = grad_slot(W)
    assert not acc and buf.data_ptr() != W.data_ptr() and buf.shape == W.shape


@pytest.mark.parametrize("order", [(0, 1, 2), (2, 0, 1)])
def test_chain_laid_out_back_to_back(order):
    from ured_hip.node import fused_rows
    ws = [torch.nn.Parameter(torch.randn(16, 16)) for _ in range(3)]
    other = torch.nn.Parameter(torch.randn(7))
    for w in ws:
        w._ured_chain = tuple(ws)
    params = [other] + [ws[i] for i in order]        # chain members in any optimizer order
    opt = FlatAdam(params, [params], lr=0.0)
    for p in params:
        p.grad = torch.zeros_like(p)
    opt.prepare()
    fused = fused_rows(ws)
    assert fused is not None and fused.shape == (48, 16)
    assert torch.equal(fused, torch.cat([w.detach() for w in ws]))


def test_post_accumulate_hook_sees_the_complete_sum_once():
    """The ownership argument of the in-kernel accumulation ("Gradient buffers"): the
    parameter's AccumulateGrad node has one input edge per use, so it runs ONCE, after every
    use's backward has run; the first claim handed it a defined tensor (the flat view), so it is
    scheduled on the device queue like any other node. The post-accumulate hook that issues a
    data-parallel bucket's all-reduce (engine/dp.py) therefore fires once per backward, on the
    flat view itself, with both uses' contributions already in it."""
    W, V, opt, x = _setup()
    x2 = torch.randn(4, 3)
    seen = []
    W.register_post_accumulate_grad_hook(lambda p: seen.append((p.grad.data_ptr(), p.grad.clone())))
    opt.zero_grad(set_to_none=True)
    y = _Lin.apply(x, W)
    (_Lin.apply(x2, W).sum() + y.sum()).backward()
    assert len(seen) == 1
    ptr, val = seen[0]
    assert ptr == _view(opt, W).data_ptr()
    torch.testing.assert_close(val, torch.ones(4, 5).t() @ x + torch.ones(4, 5).t() @ x2)


def test_accumulated_view_replaced_by_autograd_raises():
    """Guard of the accumulate contract: a non-HIP producer of the same parameter's gradient
    between two HIP uses makes autograd sum out of place, so a later in-kernel add lands in a
    tensor autograd no longer holds; gather_grads() raises instead of losing it."""
    W, V, opt, x = _setup()
    x2, x3 = torch.randn(4, 3), torch.randn(4, 3)
    opt.zero_grad(set_to_none=True)
    a = _Lin.apply(x, W)            # backward runs last: claims the view with accumulate=True
    b = x2 @ W.t()                  # an ordinary op: a fresh gradient tensor
    c = _Lin.apply(x3, W)           # backward runs first: claims the view
    (a.sum() + b.sum() + c.sum()).backward()
    with pytest.raises(RuntimeError, match="replaced by autograd"):
        opt.gather_grads()
