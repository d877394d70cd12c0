"""Part bookkeeping on the device (engine/train.py:103-136 get_part helpers): the HIP
segment AABB (ured_seg_aabb) vs compute_aabbox (dataset/dataset_utils.py:77-85) applied
per part on the CPU — bit-exact (min / max are exact, then the same two fp32 ops)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _aabb_ref(v):
    lo, hi = v.min(0).values, v.max(0).values
    return torch.cat([(lo + hi) / 2.0, (hi - lo) / 2.0])


@pytest.mark.parametrize("B,N,P,kmax", [(16, 2048, 16, 4), (3, 700, 16, 16), (2, 5, 8, 8)])
def test_part_aabb_bitexact(dev, B, N, P, kmax):
    from ured_hip.ops import build_parts, part_aabb
    g = torch.Generator().manual_seed(B * N + P)
    x = (torch.rand(B, N, 3, generator=g) * 2 - 1)
    labels = torch.randint(0, kmax, (B, N), generator=g)
    parts = build_parts(labels.to(dev), x.to(dev), P)
    got = part_aabb(parts).cpu()
    for b in range(B):
        present = sorted(set(labels[b].tolist()))
        for slot in range(P):
            if slot < len(present):
                exp = _aabb_ref(x[b][labels[b] == present[slot]])
            else:
                exp = torch.zeros(6)
            assert torch.equal(got[b, slot], exp), (b, slot)


def test_part_aabb_rejects_cpu():
    from ured_hip.ops import PartBatch, part_aabb
    pb = PartBatch(x_sorted=torch.zeros(1, 4, 3), off=torch.zeros(2, dtype=torch.int32), max_parts=1)
    with pytest.raises(RuntimeError):
        part_aabb(pb)


def test_get_shape_hip_matches_bmm(dev):
    """get_shape's HIP GEMV (ured_get_shape_fwd/bwd) vs the float64 torch.bmm of the reference
    formula (dataset_utils.py:691-726), values and the gradient w.r.t. the params; deterministic."""
    from dataset.dataset_utils import get_shape
    g = torch.Generator().manual_seed(0)
    B, P, R = 4, 16, 3 * 1024
    A = torch.randn(B, P, R, 6, generator=g).to(dev)
    prm = torch.randn(B, P, 6, generator=g).to(dev).requires_grad_(True)
    dflt = torch.randn(B, P, 6, generator=g).to(dev)
    out = get_shape(A, prm, dflt, 0.1)
    p64 = (0.1 * prm.detach().double() + dflt.double()).view(B * P, 6, 1)
    ref = torch.bmm(A.double().view(B * P, R, 6), p64).view(B, P, -1, 3)
    torch.testing.assert_close(out.double(), ref, rtol=1e-5, atol=1e-5)
    go = torch.randn(out.shape, generator=g).to(dev)
    out.backward(go)
    gref = 0.1 * torch.bmm(A.double().view(B * P, R, 6).transpose(1, 2), go.double().view(B * P, R, 1)).view(B, P, 6)
    torch.testing.assert_close(prm.grad.double(), gref, rtol=1e-4, atol=1e-4)
    g1 = prm.grad.clone()
    prm.grad = None
    get_shape(A, prm, dflt, 0.1).backward(go)
    assert torch.equal(prm.grad, g1)


@pytest.mark.parametrize("with_dflt", [True, False])
def test_get_shape_src_equals_gathered(dev, with_dflt):
    """The training step's get_shape_src (matrices read in place by source label, the parameter
    mul / add in-kernel) == get_shape over the gathered matrices, bitwise, values and gradient;
    negative labels index from the end (python indexing, dataset_utils.py:800-805)."""
    from dataset.dataset_utils import get_shape, get_shape_src, get_source_info
    from train_utils.load_sources import SourceDB
    g = torch.Generator().manual_seed(3)
    S, n, B, P = 40, 512, 4, 16
    mats = torch.randn(S, 3 * n, 6, generator=g)
    db = SourceDB(torch.randn(S, n, 3, generator=g), mats, torch.randn(S, 6, generator=g),
                  torch.randint(0, 4, (S,), generator=g), dev)
    labels = torch.randint(-S, S, (B, P), generator=g).to(dev)
    prm = torch.randn(B, P, 6, generator=g).to(dev)
    dflt = torch.randn(B, P, 6, generator=g).to(dev) if with_dflt else None
    go = torch.randn(B, P, n, 3, generator=g).to(dev)
    a = prm.clone().requires_grad_(True)
    out = get_shape_src(db, labels, a, dflt, 0.3)
    out.backward(go)
    b = prm.clone().requires_grad_(True)
    A = get_source_info(labels, db, want=(True, False, False))[0]
    ref = get_shape(A, b, dflt, 0.3)
    ref.backward(go)
    assert torch.equal(out, ref)
    assert torch.equal(a.grad, b.grad)


@pytest.mark.parametrize("B,N,P,C,kmax", [(16, 2048, 16, 512, 4), (3, 700, 16, 6, 16), (2, 5, 8, 3, 8)])
def test_part_rows_matches_separate_ops(dev, B, N, P, C, kmax):
    """PartRowsFn (gather by part label + per-part sums, one-pass HIP backward) vs the separate
    ops it replaces (permute_rows + segment_sum, autograd's index_select / add / gather):
    forward and backward bit-identical (the backward's one add is commutative)."""
    from ured_hip.ops import build_parts, part_rows, permute_rows, segment_sum
    g = torch.Generator().manual_seed(B * N + C)
    x = torch.randn(B, N, C, generator=g).to(dev)
    labels = torch.randint(0, kmax, (B, N), generator=g).to(dev)
    parts = build_parts(labels, torch.randn(B, N, 3, generator=g).to(dev), P)
    gs = torch.randn(B * N, C, generator=g).to(dev)
    gp = torch.randn(B * P, C, generator=g).to(dev)
    for use in ((True, True), (True, False), (False, True)):
        a = x.clone().requires_grad_(True)
        xs, sums = part_rows(a, parts)
        b = x.clone().requires_grad_(True)
        xs2 = permute_rows(b, parts.perm, parts.inv_perm).reshape(B * N, C)
        sums2 = segment_sum(xs2, parts.off, parts.gid)
        assert torch.equal(xs, xs2) and torch.equal(sums, sums2)
        xs_g = xs if use[0] else xs.detach()
        sums_g = sums if use[1] else sums.detach()
        outs = [t for t, u in ((xs_g, use[0]), (sums_g, use[1])) if u]
        grads = [t for t, u in ((gs, use[0]), (gp, use[1])) if u]
        torch.autograd.backward(outs, grads)
        outs2 = [t for t, u in ((xs2, use[0]), (sums2, use[1])) if u]
        torch.autograd.backward(outs2, grads)
        assert torch.equal(a.grad, b.grad), (a.grad - b.grad).abs().max().item()


@pytest.mark.parametrize("B,N,P,C,kmax", [(16, 2048, 16, 512, 4), (3, 700, 16, 6, 16)])
def test_part_rows_alias_gradient(dev, B, N, P, C, kmax):
    """part_rows(alias=True): the third output is x itself (same values, same storage) and the
    gradient reaching it is added inside the regrouping's backward pass — equal, bitwise, to
    autograd's own sum when the second consumer reads x directly."""
    from ured_hip.ops import build_parts, part_rows
    g = torch.Generator().manual_seed(B + N + C)
    x = torch.randn(B, N, C, generator=g).to(dev)
    labels = torch.randint(0, kmax, (B, N), generator=g).to(dev)
    parts = build_parts(labels, torch.randn(B, N, 3, generator=g).to(dev), P)
    gs, gp = torch.randn(B * N, C, generator=g).to(dev), torch.randn(B * P, C, generator=g).to(dev)
    gx = torch.randn(B, N, C, generator=g).to(dev)
    a = x.clone().requires_grad_(True)
    xs, sums, xa = part_rows(a, parts, alias=True)
    assert xa.data_ptr() == a.data_ptr() and torch.equal(xa, a)
    torch.autograd.backward([xs, sums, xa * 1.0], [gs, gp, gx])
    b = x.clone().requires_grad_(True)
    xs2, sums2 = part_rows(b, parts)
    torch.autograd.backward([xs2, sums2, b * 1.0], [gs, gp, gx])
    assert torch.equal(a.grad, b.grad), (a.grad - b.grad).abs().max().item()
    c = x.clone().requires_grad_(True)                  # alias output unused: no third gradient
    xs3, sums3, _ = part_rows(c, parts, alias=True)
    torch.autograd.backward([xs3, sums3], [gs, gp])
    d = x.clone().requires_grad_(True)
    xs4, sums4 = part_rows(d, parts)
    torch.autograd.backward([xs4, sums4], [gs, gp])
    assert torch.equal(c.grad, d.grad)


@pytest.mark.parametrize("B,N,P,gaps", [(3, 257, 16, True), (16, 2048, 16, False), (2, 5000, 32, True), (1, 7, 16, True)])
def test_build_parts_kernel_equals_composed(dev, B, N, P, gaps):
    """ured_build_parts (one launch: stable counting sort, slot tables, boxes, param_def) == the
    composed torch form (scatter_add / cumsum / stable sort / gathers / ured_seg_aabb) field by
    field, bitwise; absent labels (gaps) included."""
    from ured_hip.ops import build_parts, build_parts_composed, part_aabb
    g = torch.Generator().manual_seed(B * 1000 + N)
    hi = P if not gaps else P - 3
    labels = torch.randint(0, hi, (B, N), generator=g)
    if gaps:
        labels[labels == 2] = 5                     # label 2 absent everywhere
    x = torch.randn(B, N, 3, generator=g).to(dev)
    a = build_parts(labels.to(dev), x, P)
    c = build_parts_composed(labels.to(dev), x, P)
    for f in ("x_sorted", "perm", "inv_perm", "gid", "off", "counts", "k", "mask", "rank_of_label", "present"):
        ta, tc = getattr(a, f), getattr(c, f)
        assert ta.dtype == tc.dtype and ta.shape == tc.shape, f
        assert torch.equal(ta, tc), f
    assert torch.equal(a.aabb, part_aabb(c))
    pd = torch.gather(part_aabb(c), 1, c.rank_of_label.clamp(min=0).unsqueeze(-1).expand(-1, -1, 6))
    pd = pd * c.present.unsqueeze(-1).float()
    assert torch.equal(a.param_def, pd)
