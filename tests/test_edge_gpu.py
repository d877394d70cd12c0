"""Edge layers (K <= 4) of ured_gemm: the streaming forward + BN-statistics kernel and the
streaming dgrad + BN-backward kernel (csrc/mlp.hip fwd_small_stats / dgrad_small_bnbwd) against
float64 torch restatements of the GEMM epilogues they replace (EPI_FWD / EPI_BNBWD partials per
128-row block)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K(dev):
    from ured_hip import kernels
    return kernels


def _blocks(M):
    return (M + 127) // 128


@pytest.mark.parametrize("M,N,Kd,relu", [(32768, 64, 3, False), (1000, 32, 3, True), (300, 256, 4, False),
                                         (129, 3, 1, True), (4096, 128, 2, False)])
def test_fwd_small_stats(K, dev, M, N, Kd, relu):
    g = torch.Generator(device=dev).manual_seed(M + N)
    X = torch.randn(M, Kd, device=dev, generator=g)
    W = torch.randn(N, Kd, device=dev, generator=g)
    b = torch.randn(N, device=dev, generator=g)
    Y = torch.empty(M, N, device=dev)
    ws = torch.empty(_blocks(M), 2, N, device=dev)
    K.gemm(M, N, Kd, X, Kd, W, Kd, Y, N, epi=K.EPI_FWD, bias=b, stat_ws=ws, stat_relu=relu)
    ref = X.double() @ W.double().t() + b.double()
    assert (Y.double() - ref).abs().max().item() <= 1e-5 * (1 + ref.abs().max().item())
    p = ref.clamp_min(0) if relu else ref
    wv = ws.view(2, N, _blocks(M))              # partial layout [2][N][blocks] (include/ured_hip.h)
    for blk in range(_blocks(M)):
        rows = p[blk * 128:(blk + 1) * 128]
        mu = rows.mean(0)
        m2 = ((rows - mu) ** 2).sum(0)
        assert torch.allclose(wv[0, :, blk].double(), mu, rtol=1e-5, atol=1e-5)
        assert torch.allclose(wv[1, :, blk].double(), m2, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("M,N,Kd,mode,gadd", [(32768, 32, 3, 1, False), (1000, 64, 3, 0, True), (300, 256, 4, 2, False),
                                              (129, 32, 1, 0, False)])
def test_dgrad_small_bnbwd(K, dev, M, N, Kd, mode, gadd):
    g = torch.Generator(device=dev).manual_seed(M + 7 * N)
    dY = torch.randn(M, Kd, device=dev, generator=g)
    W = torch.randn(Kd, N, device=dev, generator=g)          # k-major B: W[k][n]
    Yp = torch.randn(M, N, device=dev, generator=g)
    mean = torch.randn(N, device=dev, generator=g) * 0.1
    invstd = torch.rand(N, device=dev, generator=g) + 0.5
    # power-of-two scales: y * scale is exact, so the fp64 mask below equals the kernel's fp32 fma test
    scale = torch.randint(-1, 2, (N,), device=dev, generator=g).float().exp2() * \
        (torch.randint(0, 2, (N,), device=dev, generator=g).float() * 2 - 1)
    shift = torch.randint(-2, 3, (N,), device=dev, generator=g).float() * 0.25
    ga = torch.randn(M, N, device=dev, generator=g) if gadd else None
    G = torch.empty(M, N, device=dev)
    ws = torch.empty(_blocks(M), 2, N, device=dev)
    K.gemm(M, N, Kd, dY, Kd, W, N, G, N, b_kmajor=True, epi=K.EPI_BNBWD, Yp=Yp, ldy=N,
           bn=K.BNState(mean, invstd, scale, shift), bwd_res=mode, bwd_ws=ws, gadd=ga, ldg=N if gadd else 0)
    dh = dY.double() @ W.double()
    if gadd:
        dh = dh + ga.double()
    y = Yp.double()
    if mode == 1:      # ACT_RES: Conv -> ReLU -> BN
        gr, xh = dh, (y.clamp_min(0) - mean.double()) * invstd.double()
    elif mode == 2:    # ACT_BN
        gr, xh = dh, (y - mean.double()) * invstd.double()
    else:              # ACT_ENC: Conv -> BN -> ReLU
        mask = y * scale.double() + shift.double() > 0
        gr, xh = torch.where(mask, dh, torch.zeros_like(dh)), (y - mean.double()) * invstd.double()
    assert (G.double() - gr).abs().max().item() <= 1e-5 * (1 + gr.abs().max().item())
    wv = ws.view(2, N, _blocks(M))              # partial layout [2][N][blocks] (include/ured_hip.h)
    for blk in range(_blocks(M)):
        sl = slice(blk * 128, (blk + 1) * 128)
        assert torch.allclose(wv[0, :, blk].double(), gr[sl].sum(0), rtol=1e-4, atol=1e-4)
        assert torch.allclose(wv[1, :, blk].double(), (gr[sl] * xh[sl]).sum(0), rtol=1e-4, atol=1e-4)
