"""Deterministic column reductions (ured_group_colsum_split, ured_splitk_reduce) vs float64."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K(dev):
    from ured_hip import kernels
    return kernels


@pytest.mark.parametrize("R,N,G", [(262144, 512, 1), (32768, 1024, 16), (300, 3, 1), (4096, 64, 256), (70000, 200, 7)])
def test_group_colsum_fixed_groups(K, dev, R, N, G):
    R = R // G * G
    X = torch.randn(R, N, device=dev, generator=torch.Generator(device=dev).manual_seed(R + N))
    out = K.group_colsum(X, N, G, group_rows=R // G)
    ref = X.double().view(G, R // G, N).sum(1)
    torch.testing.assert_close(out.double(), ref, rtol=1e-5, atol=1e-3)
    # deterministic
    assert torch.equal(out, K.group_colsum(X, N, G, group_rows=R // G))


def test_group_colsum_ragged_and_colsum(K, dev):
    g = torch.Generator(device=dev).manual_seed(3)
    lens = [0, 5000, 1, 20000, 777, 40000]
    off = torch.tensor(np.concatenate([[0], np.cumsum(lens)]), dtype=torch.int32, device=dev)
    R, N = int(sum(lens)), 96
    X = torch.randn(R, N, device=dev, generator=g)
    out = K.group_colsum(X, N, len(lens), off=off)
    ref = torch.stack([X[o:o + l].double().sum(0) for o, l in zip(off[:-1].tolist(), lens)])
    torch.testing.assert_close(out.double(), ref, rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(K.colsum(X).double(), X.double().sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("splits,M,N", [(256, 3, 32), (8, 1024, 1024), (37, 50, 7)])
def test_splitk_reduce(K, dev, splits, M, N):
    g = torch.Generator(device=dev).manual_seed(splits)
    ws = torch.randn(splits, M, N, device=dev, generator=g)
    out = torch.full((M, N + 5), 2.0, device=dev)
    K.splitk_reduce(ws, splits, M, N, out, N + 5, accumulate=True)
    ref = ws.double().sum(0) + 2.0
    torch.testing.assert_close(out[:, :N].double(), ref, rtol=1e-5, atol=1e-4)
    assert torch.all(out[:, N:] == 2.0)
