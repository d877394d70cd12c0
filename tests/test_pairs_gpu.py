"""Offline pseudo-label path: fused DCD kernel (ured_dcd) and the
batched all-pairs generator vs the oracle / the reference's calc_dcd golden vectors."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import dcd_ref

pytestmark = pytest.mark.gpu

TOL = 2e-6   # fp32 means of ~1e3 terms in a different (fixed) order; values ~1e-2..1


def test_calc_dcd_matches_reference_golden(dev):
    from chamfer3D.model_utils import calc_dcd
    g = np.load(os.path.join(GOLDEN, "dcd.npz"), allow_pickle=False)
    for name in ("r3x300x200", "r2x1024x1024", "r4x64x512"):
        x, gt = torch.from_numpy(g[name + "/x"]).to(dev), torch.from_numpy(g[name + "/gt"]).to(dev)
        for nr in (0, 1):
            loss, cd_p, cd_t = calc_dcd(x, gt, non_reg=bool(nr))
            tag = f"{name}/nr{nr}"
            np.testing.assert_allclose(loss.cpu().numpy(), g[tag + "/loss"], rtol=0, atol=TOL)
            np.testing.assert_allclose(cd_p.cpu().numpy(), g[tag + "/cd_p"], rtol=0, atol=TOL)
            np.testing.assert_allclose(cd_t.cpu().numpy(), g[tag + "/cd_t"], rtol=0, atol=TOL)
        loss, _, _ = calc_dcd(x, gt, alpha=200, n_lambda=2)
        np.testing.assert_allclose(loss.cpu().numpy(), g[name + "/a200l2/loss"], rtol=0, atol=TOL)


def test_calc_dcd_grad_path_equals_fused(dev):
    """With autograd on, calc_dcd keeps the differentiable torch tail; same values."""
    from chamfer3D.model_utils import calc_dcd
    r = np.random.Generator(np.random.PCG64(8))
    x = torch.from_numpy(r.random((3, 500, 3), dtype=np.float32)).to(dev)
    gt = torch.from_numpy(r.random((3, 700, 3), dtype=np.float32)).to(dev)
    with torch.no_grad():
        fused = calc_dcd(x, gt)
    xg = x.clone().requires_grad_(True)
    res = calc_dcd(xg, gt)
    res[0].sum().backward()
    assert xg.grad is not None and torch.isfinite(xg.grad).all()
    for a, b in zip(fused, res):
        torch.testing.assert_close(a, b.detach(), rtol=0, atol=TOL)


@pytest.mark.parametrize("n_pts,n_clouds,chunk", [(256, 24, 64), (1024, 9, 16384)])
def test_pair_rows_vs_oracle(dev, n_pts, n_clouds, chunk):
    from engine.generate_pair import PairGenerator, connect_matrix, normalize_pts
    r = np.random.Generator(np.random.PCG64(n_pts))
    pts = np.stack([normalize_pts(r.random((n_pts, 3), dtype=np.float32) ** 2) for _ in range(n_clouds)])
    gen = PairGenerator(torch.from_numpy(pts).to(dev), chunk_pairs=chunk)
    rows = gen.rows(range(n_clouds))
    ref = dcd_ref.pair_rows(pts)
    for i in range(n_clouds):
        for k in range(3):
            np.testing.assert_allclose(rows[i][k], ref[i][k], rtol=0, atol=TOL)
    m, mr = connect_matrix(rows, n_clouds), dcd_ref.connect_matrix(ref, n_clouds)
    np.testing.assert_allclose(m, mr, rtol=0, atol=2 * TOL)
    # deterministic: a second pass is bitwise identical
    rows2 = gen.rows([0, n_clouds - 1])
    np.testing.assert_array_equal(rows2[0][0], rows[0][0])


def test_dcd_rejects_oversize(dev):
    from ured_hip import _lib
    from ured_hip import nn as unn
    d = torch.zeros(1, 9000, device=dev)
    i = torch.zeros(1, 9000, device=dev, dtype=torch.int32)
    with pytest.raises(_lib.UredError, match="exceeds"):
        unn.dcd(d, i, d, i)
