"""Loss drop-ins (ragged HIP chamfer) vs the oracle's per-sample loops."""
import numpy as np
import pytest
import torch

from oracle import nn_ref, ured_ref

pytestmark = pytest.mark.gpu


def _case(B=3, S_parts=16, N=700, ks=(4, 1, 16), seed=0):
    g = torch.Generator().manual_seed(seed)
    S = S_parts * 1024
    out = torch.rand(B, S, 3, generator=g) - 0.5
    x = torch.rand(B, N, 3, generator=g) - 0.5
    labels = torch.stack([torch.randint(0, k, (N,), generator=g) for k in ks])
    for b, k in enumerate(ks):      # every label present (contiguous 0..k-1, as get_labels assumes)
        labels[b, :k] = torch.arange(k)
    mask = torch.zeros(B, S_parts)
    for b, k in enumerate(ks):
        mask[b, :k] = 1
    part_x = [[x[b, labels[b] == i] for i in range(k)] for b, k in enumerate(ks)]
    return out, x, labels, mask, part_x


def test_compute_cm_loss_vs_oracle(dev):
    from loss.chamfer_loss import compute_cm_loss
    from ured_hip.ops import build_parts
    out, x, labels, mask, part_x = _case()
    ref_full, ref_part = ured_ref.compute_cm_loss(out, x, part_x, mask)
    o = out.to(dev).requires_grad_(True)
    parts = build_parts(labels.to(dev), x.to(dev), 16)
    full, part = compute_cm_loss(o, x.to(dev), parts, mask.to(dev))
    assert abs(full.item() - ref_full.item()) <= 1e-6 * abs(ref_full.item())
    assert abs(part.item() - ref_part.item()) <= 1e-6 * abs(ref_part.item())
    # the reference's list-of-lists part_x form gives the same numbers
    full2, part2 = compute_cm_loss(out.to(dev), x.to(dev), [[p.to(dev) for p in pl] for pl in part_x], mask.to(dev))
    assert abs(full2.item() - full.item()) <= 1e-7 * abs(full.item())
    assert abs(part2.item() - part.item()) <= 1e-7 * abs(part.item())
    # gradient wrt the deformed shape
    (30 * full + part).backward()
    orr = out.clone().requires_grad_(True)
    rf, rp = ured_ref.compute_cm_loss(orr, x, part_x, mask)
    (30 * rf + rp).backward()
    np.testing.assert_allclose(o.grad.cpu().numpy(), orr.grad.numpy(), rtol=1e-4, atol=1e-9)


def test_unmasked_and_batch_reduction(dev):
    from loss.chamfer_loss import compute_cm_loss, chamfer_distance2
    g = torch.Generator().manual_seed(3)
    a, b = torch.rand(2, 300, 3, generator=g), torch.rand(2, 200, 3, generator=g)
    got = compute_cm_loss(a.to(dev), b.to(dev), None, batch_reduction=None).cpu()
    ref = ured_ref.chamfer_distance2(a, b)
    np.testing.assert_allclose(got.numpy(), ref.numpy(), rtol=1e-6)
    np.testing.assert_allclose(chamfer_distance2(a.to(dev), b.to(dev)).cpu().numpy(), ref.numpy(), rtol=1e-6)


def test_residual_retrieval_loss(dev):
    from loss.basic_loss import residual_retrieval_loss, knn_points
    out, x, labels, mask, _ = _case(seed=5)
    g = torch.Generator().manual_seed(6)
    res = torch.randn(x.shape, generator=g) * 0.01
    r1, r2 = ured_ref.residual_retrieval_loss(x, out, res, mask)
    g1, g2 = residual_retrieval_loss(x.to(dev), out.to(dev), res.to(dev), mask.to(dev))
    assert abs(g1.item() - r1.item()) <= 1e-6 * abs(r1.item())
    assert abs(g2.item() - r2.item()) <= 1e-6 * abs(r2.item())
    d, i, nn = knn_points(x.to(dev), out.to(dev)[:, :4096], K=1, return_nn=True)
    rd, ri = nn_ref.nn_dir(x[0].numpy(), out[0, :4096].numpy())
    np.testing.assert_array_equal(i[0, :, 0].cpu().numpy(), ri)
    np.testing.assert_array_equal(d[0, :, 0].cpu().numpy(), rd)


def test_calc_cd_dcd_fscore(dev):
    from chamfer3D.model_utils import calc_cd, calc_dcd
    from chamfer3D.dist_chamfer_3D import chamfer_3DDist
    g = torch.Generator().manual_seed(9)
    out, gt = torch.rand(2, 400, 3, generator=g), torch.rand(2, 256, 3, generator=g)
    d1, d2, i1, i2 = nn_ref.nn_fwd(gt.numpy(), out.numpy())       # calc_cd evaluates cham(gt, output)
    d1, d2 = torch.from_numpy(d1).double(), torch.from_numpy(d2).double()
    cd_p = (d1.sqrt().mean(1) + d2.sqrt().mean(1)) / 2
    cd_t = d1.mean(1) + d2.mean(1)
    r = calc_cd(out.to(dev), gt.to(dev), calc_f1=True)
    np.testing.assert_allclose(r[0].cpu().numpy(), cd_p.numpy(), rtol=1e-5)
    np.testing.assert_allclose(r[1].cpu().numpy(), cd_t.numpy(), rtol=1e-5)
    # DCD restated from model_utils.py:13-51 on the oracle's NN
    i1l, i2l = torch.from_numpy(i1).long(), torch.from_numpy(i2).long()
    c1 = torch.zeros(2, 400).scatter_add_(1, i1l, torch.ones(2, 256)).gather(1, i1l)
    c2 = torch.zeros(2, 256).scatter_add_(1, i2l, torch.ones(2, 400)).gather(1, i2l)
    l1 = (1 - torch.exp(-d1 * 1000) * (c1.double() + 1e-6) ** -1 * (256 / 400)).mean(1)
    l2 = (1 - torch.exp(-d2 * 1000) * (c2.double() + 1e-6) ** -1 * (400 / 256)).mean(1)
    dcd = calc_dcd(out.to(dev), gt.to(dev))[0].cpu()
    np.testing.assert_allclose(dcd.numpy(), ((l1 + l2) / 2).numpy(), rtol=1e-5)
    dd1, dd2, ii1, ii2 = chamfer_3DDist()(out.to(dev), gt.to(dev))
    assert ii1.dtype == torch.int32 and dd1.shape == (2, 400)


def test_cm_loss_pair_equals_two_calls(dev):
    """compute_cm_loss_pair (chamfer + symmetric chamfer in one launch per family) equals the two
    compute_cm_loss calls: the NN results are per segment (identical); only torch's row
    reductions over a [2B, .] instead of a [B, .] tensor and the gradient-accumulation grouping
    may round differently (1 ulp)."""
    from dataset.dataset_utils import get_symmetric
    from loss.chamfer_loss import compute_cm_loss, compute_cm_loss_pair
    from ured_hip.ops import build_parts
    g = torch.Generator().manual_seed(3)
    B, S, N, P = 4, 16 * 256, 512, 16
    out0 = torch.rand(B, S, 3, generator=g).to(dev)
    x = torch.rand(B, N, 3, generator=g).to(dev)
    k = torch.tensor([3, 1, 16, 5])
    labels = torch.stack([(torch.arange(N) * int(kk)) // N for kk in k]).to(dev)
    parts = build_parts(labels, x, P)
    a = out0.clone().requires_grad_(True)
    b = out0.clone().requires_grad_(True)
    (f1, p1), (f2, p2) = compute_cm_loss_pair(a, get_symmetric(a), x, parts, parts.mask, np_per_part=256)
    r1 = compute_cm_loss(b, x, parts, parts.mask, np_per_part=256)
    r2 = compute_cm_loss(get_symmetric(b), x, parts, parts.mask, np_per_part=256)
    for u, v in ((f1, r1[0]), (p1, r1[1]), (f2, r2[0]), (p2, r2[1])):
        torch.testing.assert_close(u, v, rtol=1e-6, atol=0)
    (30 * f1 + p1 + 30 * f2).backward()
    (30 * r1[0] + r1[1] + 30 * r2[0]).backward()
    torch.testing.assert_close(a.grad, b.grad, rtol=1e-6, atol=1e-6 * float(b.grad.abs().max()))


def test_residual_loss_with_chamfer_indices(dev):
    """residual_retrieval_loss fed the chamfer full family's x -> out indices equals its own
    knn_points query (the same NN primitive, same direction, same valid lengths)."""
    from loss.basic_loss import residual_retrieval_loss
    from loss.chamfer_loss import compute_cm_loss
    from ured_hip.ops import build_parts
    g = torch.Generator().manual_seed(5)
    B, S, N, P = 3, 16 * 256, 500, 16
    out = torch.rand(B, S, 3, generator=g).to(dev)
    x = torch.rand(B, N, 3, generator=g).to(dev)
    r = (torch.rand(B, N, 3, generator=g) * 0.1).to(dev)
    k = torch.tensor([2, 7, 16])
    labels = torch.stack([(torch.arange(N) * int(kk)) // N for kk in k]).to(dev)
    parts = build_parts(labels, x, P)
    _, _, idx = compute_cm_loss(out, x, parts, parts.mask, np_per_part=256, return_idx=True)
    a = residual_retrieval_loss(x, out, r, parts.mask, np_per_part=256)
    b = residual_retrieval_loss(x, out, r, parts.mask, np_per_part=256, nn_idx=idx)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
