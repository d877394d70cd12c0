"""PointNetEncoder drop-in on the HIP chain vs the reference's own outputs
(tests/golden/pointnet.npz) — forward (training-mode BN), backward of the seeded loss,
running statistics — and eval mode vs the CPU oracle.

Tolerances (fp32 MFMA sums in another order than the CPU conv; BN divides by per-channel
std, max-pool picks one row): outputs and trans 2e-4 of the tensor's max magnitude,
gradients 2e-3 of max magnitude (sampled entries for large tensors, norms 1e-3 relative),
running statistics 1e-4 — each measured against the float64 oracle and relaxed to 4x the
reference's own fp32 error against it where that is larger (training-mode BN over B = 2..4
clouds in the STN heads amplifies fp32 rounding in the reference too).
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import pointnet_ref

pytestmark = pytest.mark.gpu
G = np.load(os.path.join(GOLDEN, "pointnet.npz"))


def close(got, ref, rel, name, truth=None):
    """max|got - ref| <= rel * max|ref|; with `truth` (the float64 oracle) the bound is
    max(that, 4 x the reference's own fp32 error vs float64) — PointNet's BatchNorm over a few
    clouds (bn4/bn5 see B rows) amplifies fp32 rounding, in the reference as much as here."""
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    assert got.shape == ref.shape, (name, got.shape, ref.shape)
    scale = max(np.abs(ref).max(), 1e-6)
    if truth is not None:
        truth = np.asarray(truth, dtype=np.float64)
        err, ref_err = np.abs(got - truth).max(), np.abs(ref - truth).max()
        assert err <= max(rel * scale, 4.0 * ref_err), \
            f"{name}: err vs float64 {err:.3e} > max({rel:.1e} * {scale:.3e}, 4 * reference fp32 err {ref_err:.3e})"
        return
    err = np.abs(got - ref).max()
    assert err <= rel * scale, f"{name}: max err {err:.3e} > {rel:.1e} * {scale:.3e}"


def _bias_before_bn(k):
    leaf = k.split(".")[-2:]
    return leaf[1] == "bias" and leaf[0] in ("conv1", "conv2", "conv3", "fc1", "fc2")


def _oracle64(ci):
    """Float64 oracle step of case ci: outputs, loss and every gradient."""
    name, B, D, N, gf, ft = pointnet_ref.CASES[ci]
    P = {k: (v.double().requires_grad_(True) if v.dtype.is_floating_point and "running" not in k else v)
         for k, v in pointnet_ref.make_params(D, ft, seed=10 + ci).items()}
    x = torch.from_numpy(G[f"{name}/x"]).double().requires_grad_(True)
    out, trans, tf = pointnet_ref.pointnet_forward(P, x, gf, ft)
    loss = pointnet_ref.case_loss(out, trans, tf, rng_seed=1000 + ci)
    loss.backward()
    T = {"out": out.detach(), "trans": trans.detach(), "dx": x.grad}
    if tf is not None:
        T["trans_feat"] = tf.detach()
    for k, v in P.items():
        if isinstance(v, torch.Tensor) and v.grad is not None:
            T["grad/" + k] = v.grad.reshape(-1)
    return T


@pytest.mark.parametrize("ci", range(len(pointnet_ref.CASES)))
def test_pointnet_train_step_vs_reference(dev, ci):
    from network.pointnet.pointnet_utils import PointNetEncoder
    name, B, D, N, gf, ft = pointnet_ref.CASES[ci]
    T = _oracle64(ci)
    m = PointNetEncoder(global_feat=gf, feature_transform=ft, channel=D)
    m.load_state_dict(pointnet_ref.make_params(D, ft, seed=10 + ci), strict=True)
    m.to(dev).train()
    x = torch.from_numpy(G[f"{name}/x"]).to(dev).requires_grad_(True)
    out, trans, tf = m(x)
    loss = pointnet_ref.case_loss(out, trans, tf, rng_seed=1000 + ci)
    loss.backward()
    close(out.detach().cpu(), G[f"{name}/out"], 2e-4, "out", T["out"])
    close(trans.detach().cpu(), G[f"{name}/trans"], 2e-4, "trans", T["trans"])
    if ft:
        close(tf.detach().cpu(), G[f"{name}/trans_feat"], 2e-4, "trans_feat", T["trans_feat"])
    ref_loss = float(G[f"{name}/loss"])
    assert abs(loss.item() - ref_loss) <= 1e-4 * abs(ref_loss) + 1e-4
    close(x.grad.cpu(), G[f"{name}/dx"], 2e-3, "dx", T["dx"])
    for k, p in m.named_parameters():
        g = p.grad.detach().cpu().numpy().reshape(-1)
        t64 = T["grad/" + k].numpy()
        if _bias_before_bn(k):
            # a bias followed by training-mode BN has a zero gradient: both sides are rounding
            # noise, bounded relative to the same layer's weight gradient
            wk = k[:-len("bias")] + "weight"
            wref = G[f"{name}/grad/{wk}"] if f"{name}/grad/{wk}" in G else G[f"{name}/gval/{wk}"]
            assert np.abs(g).max() <= 2e-3 * np.abs(wref).max(), k
        elif f"{name}/grad/{k}" in G:
            close(g, G[f"{name}/grad/{k}"], 2e-3, k, t64)
        else:
            ref_n = float(G[f"{name}/gnorm/{k}"])
            n64 = float(np.linalg.norm(t64))
            assert abs(np.linalg.norm(g.astype(np.float64)) - n64) <= max(1e-3 * ref_n, 4 * abs(ref_n - n64)), k
            idx = G[f"{name}/gidx/{k}"]
            close(g[idx], G[f"{name}/gval/{k}"], 2e-3, k, t64[idx])
    for k, v in m.state_dict().items():
        if f"{name}/state/{k}" in G:
            close(v.cpu(), G[f"{name}/state/{k}"], 1e-4, k)


def test_pointnet_eval_mode_vs_oracle(dev):
    """Eval BN (running statistics) on the HIP chain vs the oracle with the same running stats."""
    import torch.nn.functional as F
    from network.pointnet.pointnet_utils import PointNetEncoder
    P = pointnet_ref.make_params(3, False, seed=3)
    g = torch.Generator().manual_seed(5)
    for k in list(P):
        if k.endswith("running_mean"):
            P[k] = torch.randn(P[k].shape, generator=g) * 0.1
        elif k.endswith("running_var"):
            P[k] = torch.rand(P[k].shape, generator=g) + 0.5
    m = PointNetEncoder(global_feat=False, feature_transform=False).to(dev)
    m.load_state_dict(P, strict=True)
    m.eval()
    x = torch.rand(2, 3, 256, generator=g) * 2 - 1
    with torch.no_grad():
        out, trans, _ = m(x.to(dev))
    Pe = {k: v.double() if v.dtype.is_floating_point else v for k, v in P.items()}
    orig = pointnet_ref._bn_train
    try:
        pointnet_ref._bn_train = lambda t, Q, pre: F.batch_norm(t, Q[pre + "running_mean"], Q[pre + "running_var"],
                                                                Q[pre + "weight"], Q[pre + "bias"], training=False,
                                                                eps=pointnet_ref.EPS)
        ro, rt, _ = pointnet_ref.pointnet_forward(Pe, x.double(), False, False)
    finally:
        pointnet_ref._bn_train = orig
    close(trans.cpu(), rt, 2e-4, "trans")
    close(out.cpu(), ro, 2e-4, "out")
