"""PointNetEncoder: the CPU oracle (oracle/pointnet_ref.py) pinned against the
reference's own outputs (tests/golden/pointnet.npz, make_golden_pointnet.py), and the drop-in
module's state_dict keys. CPU only."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import pointnet_ref

G = np.load(os.path.join(GOLDEN, "pointnet.npz"))


def _params_with_grad(ci, D, ft):
    P = pointnet_ref.make_params(D, ft, seed=10 + ci)
    for k, v in P.items():
        if v.dtype.is_floating_point and "running" not in k:
            v.requires_grad_(True)
    return P


@pytest.mark.parametrize("ci", range(len(pointnet_ref.CASES)))
def test_oracle_matches_reference_golden(ci):
    name, B, D, N, gf, ft = pointnet_ref.CASES[ci]
    P = _params_with_grad(ci, D, ft)
    x = torch.from_numpy(G[f"{name}/x"]).requires_grad_(True)
    out, trans, tf = pointnet_ref.pointnet_forward(P, x, gf, ft)
    loss = pointnet_ref.case_loss(out, trans, tf, rng_seed=1000 + ci)
    loss.backward()
    np.testing.assert_allclose(out.detach().numpy(), G[f"{name}/out"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(trans.detach().numpy(), G[f"{name}/trans"], rtol=1e-5, atol=1e-5)
    if ft:
        np.testing.assert_allclose(tf.detach().numpy(), G[f"{name}/trans_feat"], rtol=1e-5, atol=1e-5)
    assert abs(loss.item() - float(G[f"{name}/loss"])) <= 1e-5 * abs(float(G[f"{name}/loss"])) + 1e-5
    np.testing.assert_allclose(x.grad.numpy(), G[f"{name}/dx"], rtol=1e-4, atol=1e-5)
    for k, v in P.items():
        if v.grad is None:
            continue
        g = v.grad.numpy().reshape(-1)
        if f"{name}/grad/{k}" in G:
            ref = G[f"{name}/grad/{k}"]
            assert np.abs(g - ref).max() <= 1e-4 * max(np.abs(ref).max(), 1e-6) + 1e-6, k
        else:
            assert abs(np.linalg.norm(g) - G[f"{name}/gnorm/{k}"]) <= 1e-4 * G[f"{name}/gnorm/{k}"], k
            ref = G[f"{name}/gval/{k}"]
            got = g[G[f"{name}/gidx/{k}"]]
            assert np.abs(got - ref).max() <= 1e-4 * max(np.abs(ref).max(), 1e-6) + 1e-6, k


@pytest.mark.parametrize("ft", [False, True])
def test_dropin_state_dict_keys(ft):
    """The drop-in loads the oracle's (= the reference's, pinned by make_golden strict=True) keys strictly."""
    from network.pointnet.pointnet_utils import PointNetEncoder
    m = PointNetEncoder(global_feat=True, feature_transform=ft, channel=3)
    m.load_state_dict(pointnet_ref.make_params(3, ft, seed=0), strict=True)


def test_dropin_refuses_cpu_tensors(built):
    """No CPU fallback: the HIP chain raises on host tensors."""
    from network.pointnet.pointnet_utils import PointNetEncoder
    m = PointNetEncoder()
    with pytest.raises(RuntimeError, match="MI355X only"):
        m(torch.rand(2, 3, 128))
