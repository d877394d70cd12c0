"""HIP nearest-neighbour kernels vs the C oracle (bit-exact distances and
indices: the kernels and the oracle evaluate the same fp32 formula)."""
import numpy as np
import pytest
import torch

from oracle import nn_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def unn(dev):
    from ured_hip import nn
    return nn


def _rand(shape, seed):
    return np.random.Generator(np.random.PCG64(seed)).random(shape, dtype=np.float32)


@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("b,n,m", [(4, 100, 200), (3, 257, 129), (2, 1, 5), (1, 2048, 2048), (2, 1023, 1025),
                                   (5, 3000, 17), (1, 17, 4100), (2, 512, 512), (1, 4096, 3000), (3, 4096, 33)])
def test_dense_fwd_bitexact(unn, dev, b, n, m, fused, monkeypatch):
    monkeypatch.setattr(unn, "FUSED_MIN_PAIRS", 0 if fused else 1 << 62)
    monkeypatch.setattr(unn, "FUSED_MIN_PAIRS_SMALL_SETS", 0 if fused else 1 << 62)
    p1, p2 = _rand((b, n, 3), n), _rand((b, m, 3), m + 7)
    d1, d2, i1, i2 = unn.nn_dense(torch.from_numpy(p1).to(dev), torch.from_numpy(p2).to(dev))
    r = nn_ref.nn_fwd(p1, p2)
    np.testing.assert_array_equal(i1.cpu().numpy(), r[2])
    np.testing.assert_array_equal(i2.cpu().numpy(), r[3])
    np.testing.assert_array_equal(d1.cpu().numpy(), r[0])
    np.testing.assert_array_equal(d2.cpu().numpy(), r[1])


def test_dense_golden_distchamfer(unn, dev):
    """The reference unit test's own criterion (ChamferDistancePytorch/unit_test.py:14-35)."""
    import os
    from conftest import GOLDEN
    g = np.load(os.path.join(GOLDEN, "nn_distchamfer.npz"))
    for case in ("u4x100x200", "u3x257x129", "u2x1x5", "u1x2048x2048"):
        d1, d2, i1, i2 = unn.nn_dense(torch.from_numpy(g[case + "/p1"]).to(dev), torch.from_numpy(g[case + "/p2"]).to(dev))
        assert ((d1.cpu().numpy() - g[case + "/d1"]) ** 2).mean() + ((d2.cpu().numpy() - g[case + "/d2"]) ** 2).mean() < 1e-8
        np.testing.assert_array_equal(i1.cpu().numpy(), g[case + "/i1"])
        np.testing.assert_array_equal(i2.cpu().numpy(), g[case + "/i2"])


def test_ties_lowest_index(unn, dev):
    ax = np.linspace(0, 1, 6, dtype=np.float32)
    grid = np.stack(np.meshgrid(ax, ax, ax, indexing="ij"), -1).reshape(1, -1, 3)
    q = np.concatenate([np.full((1, 300, 3), 0.1, np.float32), _rand((1, 200, 3), 3)], 1)
    grid2 = np.concatenate([grid, grid, grid], 1)  # duplicated refs: every min is tied 3x
    for refs in (grid, grid2):
        d1, d2, i1, i2 = unn.nn_dense(torch.from_numpy(q).to(dev), torch.from_numpy(refs).to(dev))
        r = nn_ref.nn_fwd(q, refs)
        np.testing.assert_array_equal(i1.cpu().numpy(), r[2])
        np.testing.assert_array_equal(i2.cpu().numpy(), r[3])
        np.testing.assert_array_equal(d1.cpu().numpy(), r[0])


@pytest.mark.parametrize("b,n,m", [(4, 100, 200), (2, 1300, 700), (1, 2048, 2048)])
def test_dense_bwd(unn, dev, b, n, m):
    p1, p2 = _rand((b, n, 3), 11), _rand((b, m, 3), 12)
    g1, g2 = _rand((b, n), 13) - 0.5, _rand((b, m), 14) - 0.5
    a = torch.from_numpy(p1).to(dev).requires_grad_(True)
    c = torch.from_numpy(p2).to(dev).requires_grad_(True)
    d1, d2, i1, i2 = unn.nn_dense(a, c)
    (d1 * torch.from_numpy(g1).to(dev)).sum().add((d2 * torch.from_numpy(g2).to(dev)).sum()).backward()
    r = nn_ref.nn_fwd(p1, p2)
    ga, gc = nn_ref.nn_bwd(p1, p2, g1, g2, r[2], r[3])
    np.testing.assert_allclose(a.grad.cpu().numpy(), ga, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(c.grad.cpu().numpy(), gc, rtol=1e-6, atol=1e-7)
    # deterministic: a second run is bitwise identical
    a2 = a.detach().clone().requires_grad_(True)
    d1b, d2b, _, _ = unn.nn_dense(a2, c.detach())
    (d1b * torch.from_numpy(g1).to(dev)).sum().add((d2b * torch.from_numpy(g2).to(dev)).sum()).backward()
    assert torch.equal(a2.grad, a.grad)


def test_dense_outputs_allow_inplace(unn, dev):
    """dist1 / dist2 are independent allocations (as the reference's chamfer_3DDist returns them):
    an in-place op on one of them works under autograd and leaves the other and the indices
    untouched; the clamped gradient flows through the in-place op."""
    p1, p2 = _rand((2, 300, 3), 41), _rand((2, 200, 3), 42)
    a = torch.from_numpy(p1).to(dev).requires_grad_(True)
    c = torch.from_numpy(p2).to(dev).requires_grad_(True)
    d1, d2, i1, i2 = unn.nn_dense(a, c)
    assert d1.data_ptr() != d2.data_ptr() and d1._base is None and d2._base is None
    d2_before, i1_before = d2.detach().clone(), i1.clone()
    d1.clamp_(max=0.001)
    assert torch.equal(d2, d2_before) and torch.equal(i1, i1_before)
    (d1.sum() + d2.sum()).backward()
    r = nn_ref.nn_fwd(p1, p2)
    g1 = (r[0] <= 0.001).astype(np.float32)
    ga, gc = nn_ref.nn_bwd(p1, p2, g1, np.ones_like(r[1]), r[2], r[3])
    np.testing.assert_allclose(a.grad.cpu().numpy(), ga, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(c.grad.cpu().numpy(), gc, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("b,n,m", [(4, 100, 200), (2, 3000, 17), (1, 2048, 2048)])
def test_dense_bwd_set_equals_accumulate(unn, dev, b, n, m):
    """ured_nn_bwd_set (written gradients, the autograd path) == ured_nn_bwd (accumulated into
    zeroed buffers, the reference contract) bitwise, whatever the output buffers held before;
    one-direction gradients (gd2 = NULL) too."""
    from ured_hip import _lib
    p1 = torch.from_numpy(_rand((b, n, 3), 31)).to(dev)
    p2 = torch.from_numpy(_rand((b, m, 3), 32)).to(dev)
    gd1 = torch.from_numpy(_rand((b, n), 33) - 0.5).to(dev)
    gd2 = torch.from_numpy(_rand((b, m), 34) - 0.5).to(dev)
    _, _, i1, i2 = unn.nn_dense(p1, p2)
    i1, i2 = i1.contiguous(), i2.contiguous()
    for g2in in (gd2, None):
        ref1, ref2 = torch.zeros_like(p1), torch.zeros_like(p2)
        _lib.call("ured_nn_bwd", _lib.ptr(p1), _lib.ptr(p2), b, n, m, _lib.ptr(gd1), _lib.ptr(g2in),
                  _lib.ptr(i1), _lib.ptr(i2), _lib.ptr(ref1), _lib.ptr(ref2), _lib.stream_of(p1))
        out1 = torch.full_like(p1, float("nan"))
        out2 = torch.full_like(p2, float("nan"))
        _lib.call("ured_nn_bwd_set", _lib.ptr(p1), _lib.ptr(p2), b, n, m, _lib.ptr(gd1), _lib.ptr(g2in),
                  _lib.ptr(i1), _lib.ptr(i2), _lib.ptr(out1), _lib.ptr(out2), _lib.stream_of(p1))
        assert torch.equal(out1, ref1) and torch.equal(out2, ref2)


@pytest.mark.parametrize("n,m", [(3000, 5), (5000, 1), (70, 1300)])
def test_dense_bwd_degenerate(unn, dev, n, m):
    """Many queries sharing one NN (long per-point contribution lists, > one LDS tile)."""
    p1 = _rand((2, n, 3), 21)
    p2 = np.repeat(_rand((2, 1, 3), 22), m, axis=1).copy()   # m identical refs -> all map to index 0
    g1, g2 = _rand((2, n), 23) - 0.5, _rand((2, m), 24) - 0.5
    a = torch.from_numpy(p1).to(dev).requires_grad_(True)
    c = torch.from_numpy(p2).to(dev).requires_grad_(True)
    d1, d2, i1, i2 = unn.nn_dense(a, c)
    (d1 * torch.from_numpy(g1).to(dev)).sum().add((d2 * torch.from_numpy(g2).to(dev)).sum()).backward()
    r = nn_ref.nn_fwd(p1, p2)
    np.testing.assert_array_equal(i1.cpu().numpy(), r[2])
    ga, gc = nn_ref.nn_bwd(p1, p2, g1, g2, r[2], r[3])
    np.testing.assert_allclose(a.grad.cpu().numpy(), ga, rtol=1e-6, atol=1e-7)
    # up to 5000 terms summed in a different order from the scatter-form oracle
    np.testing.assert_allclose(c.grad.cpu().numpy(), gc, rtol=1e-5, atol=1e-3)


def _segs(rng, na_tot, nb_tot, nseg, max_a, max_b, allow_empty=True):
    segs, ao, bo = [], 0, 0
    for _ in range(nseg):
        al = int(rng.integers(0 if allow_empty else 1, max_a + 1))
        bl = int(rng.integers(0 if allow_empty else 1, max_b + 1))
        segs.append([ao, al, bo, bl])
        ao += al + int(rng.integers(0, 5)); bo += bl + int(rng.integers(0, 5))
    return np.array(segs, np.int32), ao, bo


@pytest.mark.parametrize("dirs", [1, 2, 3])
def test_segments_fwd_bwd(unn, dev, dirs):
    rng = np.random.Generator(np.random.PCG64(dirs))
    segs, na, nb = _segs(rng, 0, 0, 37, 3000, 1500)
    a, b = _rand((na, 3), 21), _rand((nb, 3), 22)
    ta = torch.from_numpy(a).to(dev).requires_grad_(True)
    tb = torch.from_numpy(b).to(dev).requires_grad_(True)
    ts = torch.from_numpy(segs).to(dev)
    da, ia, db, ib = unn.nn_segments(ta, tb, ts, 3000, 1500, dirs)
    r = nn_ref.nn_seg_fwd(a, b, segs, dirs)
    if dirs & 1:
        np.testing.assert_array_equal(ia.cpu().numpy(), r[1]); np.testing.assert_array_equal(da.detach().cpu().numpy(), r[0])
    if dirs & 2:
        np.testing.assert_array_equal(ib.cpu().numpy(), r[3]); np.testing.assert_array_equal(db.detach().cpu().numpy(), r[2])
    wa, wb = _rand(na, 5) - 0.5, _rand(nb, 6) - 0.5
    loss = (da * torch.from_numpy(wa).to(dev)).sum() + (db * torch.from_numpy(wb).to(dev)).sum()
    loss.backward()
    ga, gb = nn_ref.nn_seg_bwd(a, b, segs, wa if dirs & 1 else None, wb if dirs & 2 else None, r[1], r[3])
    np.testing.assert_allclose(ta.grad.cpu().numpy(), ga.reshape(-1, 3), rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(tb.grad.cpu().numpy(), gb.reshape(-1, 3), rtol=1e-6, atol=1e-7)


def test_full_size_properties(unn, dev):
    """BASELINE config-2 chamfer shape (16 x 16384 ragged vs 2048): size-independent checks
    on every query plus oracle rows on a sample."""
    B, S, N = 16, 16384, 2048
    g = torch.Generator(device="cpu").manual_seed(0)
    out = torch.rand(B, S, 3, generator=g).to(dev)
    x = torch.rand(B, N, 3, generator=g).to(dev)
    k = torch.randint(1, 17, (B,), generator=g)
    segs = torch.stack([torch.arange(B) * S, k * 1024, torch.arange(B) * N, torch.full((B,), N)], 1).int().to(dev)
    da, ia, db, ib = unn.nn_segments(out, x, segs, S, N, 3)
    for bb in range(B):
        L = int(k[bb]) * 1024
        q = out[bb, :L]
        # idx in range, reported distance equals the distance to the reported point
        assert int(ia[bb, :L].min()) >= 0 and int(ia[bb, :L].max()) < N
        r = x[bb][ia[bb, :L].long()]
        dd = ((r - q) ** 2).sum(-1)
        assert torch.allclose(dd, da[bb, :L], rtol=1e-5, atol=1e-7)
        assert int(ib[bb].max()) < L
        # untouched tail stays zero
        assert float(da[bb, L:].abs().sum()) == 0.0
    # oracle on a sample of rows
    for bb in (0, 7, 15):
        L = int(k[bb]) * 1024
        rows = slice(0, 512)
        rd, ri = nn_ref.nn_dir(out[bb, rows].cpu().numpy(), x[bb].cpu().numpy())
        np.testing.assert_array_equal(ia[bb, rows].cpu().numpy(), ri)
        np.testing.assert_array_equal(da[bb, rows].cpu().numpy(), rd)
        rd2, ri2 = nn_ref.nn_dir(x[bb, :256].cpu().numpy(), out[bb, :L].cpu().numpy())
        np.testing.assert_array_equal(ib[bb, :256].cpu().numpy(), ri2)


def test_errors_raise(unn, dev):
    from ured_hip import _lib
    with pytest.raises(RuntimeError):
        unn.nn_dense(torch.rand(2, 5, 3), torch.rand(2, 5, 3))  # CPU tensors: no fallback
    with pytest.raises(_lib.UredError):
        _lib.call("ured_nn_fwd", None, None, 1, 4, 4, 3, None, None, None, None, None)


@pytest.fixture
def fused_always(unn, monkeypatch):
    """Fused path at every size (the wrapper otherwise keeps small launches two-pass)."""
    monkeypatch.setattr(unn, "FUSED_MIN_PAIRS", 0)
    monkeypatch.setattr(unn, "FUSED_MIN_PAIRS_SMALL_SETS", 0)


@pytest.fixture
def two_pass(unn):
    """Run the wrapped block with the two-pass forward (ured_nn_fwd / ured_nn_seg_fwd)."""
    class _Ctx:
        def __enter__(self):
            unn.FUSED = False

        def __exit__(self, *a):
            unn.FUSED = True
    return _Ctx()


@pytest.mark.parametrize("b,n,m", [(8, 5000, 3000), (2, 20000, 700), (64, 1024, 1024), (3, 33, 9000)])
def test_fused_equals_two_pass(unn, dev, fused_always, two_pass, b, n, m):
    """The fused both-direction forward (several q-tiles and ref ranges per pair) is bitwise
    the two-pass kernel; small sizes are checked against the C oracle directly above."""
    g = torch.Generator(device="cpu").manual_seed(n + m)
    p1, p2 = torch.rand(b, n, 3, generator=g).to(dev), torch.rand(b, m, 3, generator=g).to(dev)
    fused = unn.nn_dense(p1, p2)
    with two_pass:
        ref = unn.nn_dense(p1, p2)
    for x, y in zip(fused, ref):
        assert torch.equal(x, y)


def test_fused_column_ties_across_tiles(unn, dev, fused_always):
    """Exact column ties between queries of different q-tiles / lanes / ref ranges: every ref
    of a lattice has several identical query copies spread over the query range; the lowest
    query index must win, as in the reference (chamfer3D.cu strict '<')."""
    ax = np.linspace(0, 1, 6, dtype=np.float32)
    grid = np.stack(np.meshgrid(ax, ax, ax, indexing="ij"), -1).reshape(-1, 3)
    rng = np.random.Generator(np.random.PCG64(5))
    q = rng.random((6000, 3), dtype=np.float32) * 0.5 + 0.25
    for pos in (100, 1500, 2900, 4100, 5700):      # copies in different tiles
        q[pos:pos + len(grid)] = grid
    refs = np.concatenate([grid, rng.random((3000, 3), dtype=np.float32)], 0)
    for qq, rr in ((q, refs), (refs, q)):
        d1, d2, i1, i2 = unn.nn_dense(torch.from_numpy(qq[None]).to(dev), torch.from_numpy(rr[None]).to(dev))
        r = nn_ref.nn_fwd(qq[None], rr[None])
        np.testing.assert_array_equal(i1.cpu().numpy(), r[2])
        np.testing.assert_array_equal(i2.cpu().numpy(), r[3])
        np.testing.assert_array_equal(d1.cpu().numpy(), r[0])
        np.testing.assert_array_equal(d2.cpu().numpy(), r[1])


def test_fused_segments_equal_two_pass(unn, dev, fused_always, two_pass):
    """Ragged families as the train step issues them (k_b*1024 vs 2048, per-part 1024 vs
    1024) plus empty pairs: fused == two-pass, bitwise."""
    rng = np.random.Generator(np.random.PCG64(9))
    segs, na, nb = _segs(rng, 0, 0, 40, 16384, 2048)
    a, b = torch.rand(na, 3).to(dev), torch.rand(nb, 3).to(dev)
    ts = torch.from_numpy(segs).to(dev)
    fused = unn.nn_segments(a, b, ts, 16384, 2048, 3)
    with two_pass:
        ref = unn.nn_segments(a, b, ts, 16384, 2048, 3)
    for x, y in zip(fused, ref):
        assert torch.equal(x, y)
