"""Fused per-point MLP (HIP, fp32 MFMA) vs the fp32 torch-CPU oracle.

Tolerances: forward outputs 2e-4 relative to the tensor's max magnitude;
gradients 2e-3 relative to max magnitude (fp32 sums over up to 10^5 points in
a different order); BN running statistics 1e-4.
"""
import numpy as np
import pytest
import torch

from oracle import ured_ref

pytestmark = pytest.mark.gpu


def close(got, ref, rel, name=""):
    got = got.detach().float().cpu()
    ref = ref.detach().float().cpu()
    assert got.shape == ref.shape, (name, got.shape, ref.shape)
    scale = max(ref.abs().max().item(), 1e-6)
    err = (got - ref).abs().max().item()
    assert err <= rel * scale, f"{name}: max err {err:.3e} > {rel:.1e} * {scale:.3e}"


@pytest.fixture(scope="module")
def K(dev):
    from ured_hip import kernels
    return kernels


@pytest.mark.parametrize("M,N,Kd", [(1000, 70, 33), (128, 128, 32), (300, 3, 32), (257, 64, 3), (4096, 1024, 64),
                                   (5000, 64, 3)])
def test_gemm_forward_store(K, dev, M, N, Kd):
    g = torch.Generator().manual_seed(M + N + Kd)
    A = torch.randn(M, Kd, generator=g)
    W = torch.randn(N, Kd, generator=g)
    b = torch.randn(N, generator=g)
    C = torch.empty(M, N, device=dev)
    K.gemm(M, N, Kd, A.to(dev), Kd, W.to(dev), Kd, C, N, bias=b.to(dev))
    close(C, A @ W.t() + b, 1e-5, "store")


@pytest.mark.parametrize("pro", [1, 2])
def test_gemm_prologue_stats(K, dev, pro):
    g = torch.Generator().manual_seed(pro)
    M, N, Kd = 777, 96, 48
    X = torch.randn(M, Kd, generator=g)
    s, t = torch.rand(Kd, generator=g) + 0.5, torch.randn(Kd, generator=g)
    W = torch.randn(N, Kd, generator=g)
    Xd = X.to(dev)
    Y = torch.empty(M, N, device=dev)
    ws = torch.empty(K.nblocks(M), 2, N, device=dev)
    K.gemm(M, N, Kd, Xd, Kd, W.to(dev), Kd, Y, N, pro_a=pro, pro_s=s.to(dev), pro_t=t.to(dev),
           epi=K.EPI_FWD, stat_ws=ws, stat_relu=(pro == 2))
    h = torch.relu(X * s + t) if pro == 1 else torch.relu(X) * s + t
    ref = h @ W.t()
    close(Y, ref, 1e-5, "fwd")
    gam, bet = torch.rand(N, generator=g) + 0.5, torch.randn(N, generator=g)
    rm, rv = torch.zeros(N, device=dev), torch.ones(N, device=dev)
    st = K.bn_fwd_finalize(ws, M, N, gam.to(dev), bet.to(dev), 1e-5, 0.1, rm, rv)
    p = torch.relu(ref) if pro == 2 else ref
    mu, var = p.double().mean(0), p.double().var(0, unbiased=False)
    close(st.mean, mu.float(), 1e-5, "mean")
    close(st.invstd, (1 / torch.sqrt(var + 1e-5)).float(), 1e-5, "invstd")
    close(rv, (0.9 + 0.1 * p.double().var(0, unbiased=True)).float(), 1e-5, "running_var")


def test_gemm_wgrad_and_dgrad(K, dev):
    g = torch.Generator().manual_seed(5)
    M, N, Kd = 20000, 200, 72
    dY = torch.randn(M, N, generator=g)
    X = torch.randn(M, Kd, generator=g)
    W = torch.randn(N, Kd, generator=g)
    dW = torch.empty(N, Kd, device=dev)
    K.wgrad(dY.to(dev), N, X.to(dev), Kd, N, Kd, M, dW, Kd)
    close(dW, dY.double().t() @ X.double(), 1e-5, "wgrad")
    dX = torch.empty(M, Kd, device=dev)
    K.gemm(M, Kd, N, dY.to(dev), N, W.to(dev), Kd, dX, Kd, b_kmajor=True)
    close(dX, dY @ W, 1e-5, "dgrad")


def test_gemm_k3_padded_views(K, dev):
    """The xyz-layer GEMMs (K = 3, zero-padded to 4 for the MFMA kernel) on strided, offset views:
    forward with batch statistics, and the k-major dgrad form."""
    g = torch.Generator().manual_seed(33)
    M, N = 9000, 96
    A = torch.randn(M, 8, generator=g)
    W = torch.randn(N, 7, generator=g)
    Y = torch.empty(M, N, device=dev)
    ws = torch.empty(K.nblocks(M), 2, N, device=dev)
    K.gemm(M, N, 3, A.to(dev), 8, W.to(dev), 7, Y, N, A_off=2, B_off=1, epi=K.EPI_FWD, stat_ws=ws)
    ref = A[:, 2:5] @ W[:, 1:4].t()
    close(Y, ref, 1e-5, "k3 fwd")
    st = K.bn_fwd_finalize(ws, M, N, torch.ones(N, device=dev), torch.zeros(N, device=dev), 1e-5, 0.1,
                           torch.zeros(N, device=dev), torch.ones(N, device=dev))
    close(st.mean, ref.double().mean(0).float(), 1e-5, "k3 fwd mean")
    Wk = torch.randn(5, N + 4, generator=g)
    dX = torch.empty(M, N, device=dev)
    K.gemm(M, N, 3, A.to(dev), 8, Wk.to(dev), N + 4, dX, N, A_off=2, B_off=N + 4 + 2, b_kmajor=True)
    close(dX, A[:, 2:5] @ Wk[1:4, 2:2 + N], 1e-5, "k3 dgrad")


@pytest.mark.parametrize("M,N,Kd", [(1000, 32, 256), (1000, 64, 64), (999, 40, 48), (4096, 64, 96), (130, 3, 64)])
def test_gemm_narrow_forward(K, dev, M, N, Kd):
    """Outputs of <= 64 columns take the 128 x 64 block tile (gemm2_kernel TN = 1); K = 33..64 also
    takes the two-stage-up-front prologue. Store form and the BN-statistics form with both
    prologues, vs float64."""
    g = torch.Generator().manual_seed(M + 7 * N + Kd)
    A = torch.randn(M, Kd, generator=g)
    W = torch.randn(N, Kd, generator=g)
    b = torch.randn(N, generator=g)
    C = torch.empty(M, N, device=dev)
    K.gemm(M, N, Kd, A.to(dev), Kd, W.to(dev), Kd, C, N, bias=b.to(dev))
    close(C, A.double() @ W.double().t() + b.double(), 1e-5, "narrow store")
    for pro in (1, 2):
        s, t = torch.rand(Kd, generator=g) + 0.5, torch.randn(Kd, generator=g)
        Y = torch.empty(M, N, device=dev)
        ws = torch.empty(K.nblocks(M), 2, N, device=dev)
        K.gemm(M, N, Kd, A.to(dev), Kd, W.to(dev), Kd, Y, N, pro_a=pro, pro_s=s.to(dev), pro_t=t.to(dev),
               epi=K.EPI_FWD, stat_ws=ws, stat_relu=(pro == 2))
        h = torch.relu(A.double() * s + t) if pro == 1 else torch.relu(A.double()) * s + t
        ref = h @ W.double().t()
        close(Y, ref, 1e-5, f"narrow fwd pro{pro}")
        st = K.bn_fwd_finalize(ws, M, N, torch.ones(N, device=dev), torch.zeros(N, device=dev), 1e-5, 0.1,
                               torch.zeros(N, device=dev), torch.ones(N, device=dev))
        p = torch.relu(ref) if pro == 2 else ref
        close(st.mean, p.mean(0).float(), 1e-5, f"narrow fwd pro{pro} mean")


@pytest.mark.parametrize("Cout,Kin,M,pro", [(32, 256, 32768, 2), (64, 64, 20000, 1), (128, 64, 9000, 1),
                                            (64, 128, 5000, 0), (40, 200, 3000, 2), (32, 256, 100, 0)])
def test_gemm_narrow_wgrad(K, dev, Cout, Kin, M, pro):
    """Weight gradients of <= 64 output rows (64-row tiles, TM = 1) and/or <= 64 columns (TN = 1),
    split-K over the points, with the wgrad prologues, vs float64; and the dgrad of the same layer
    (TN = 1 when Kin <= 64)."""
    g = torch.Generator().manual_seed(Cout + Kin + M)
    dY = torch.randn(M, Cout, generator=g)
    X = torch.randn(M, Kin, generator=g)
    s, t = torch.rand(Kin, generator=g) + 0.5, torch.randn(Kin, generator=g)
    dW = torch.empty(Cout, Kin, device=dev)
    kw = {} if pro == 0 else dict(pro=pro, pro_s=s.to(dev), pro_t=t.to(dev))
    K.wgrad(dY.to(dev), Cout, X.to(dev), Kin, Cout, Kin, M, dW, Kin, **kw)
    Xp = X.double() if pro == 0 else (torch.relu(X.double() * s + t) if pro == 1 else torch.relu(X.double()) * s + t)
    close(dW, dY.double().t() @ Xp, 1e-5, "narrow wgrad")
    W = torch.randn(Cout, Kin, generator=g)
    dX = torch.empty(M, Kin, device=dev)
    K.gemm(M, Kin, Cout, dY.to(dev), Cout, W.to(dev), Kin, dX, Kin, b_kmajor=True)
    close(dX, dY.double() @ W.double(), 1e-5, "narrow dgrad")


CFG = {"source_latent_dim": 64, "target_latent_dim": 64, "sem_latent_dim": 16, "MAX_NUM_PARTS": 16}


def _mods(dev):
    from network.simple_encoder import TargetEncoder
    from network.deformation_net import re_residual_net
    P = ured_ref.make_params(CFG, seed=3)
    tgt = TargetEncoder(64, sem_size=16)
    tgt.load_state_dict(P["target_encoder_full"], strict=True)
    src = TargetEncoder(64, is_src=True, sem_size=16)
    src.load_state_dict(P["src_encoder_all"], strict=True)
    rn = re_residual_net(128)
    rn.load_state_dict(P["recon_decoder_full"], strict=True)
    return P, tgt.to(dev).train(), src.to(dev).train(), rn.to(dev).train()


BN_FED_BIAS = ("mlp1.0.bias", "mlp1.3.bias", "mlp2.0.bias", "mlp2.3.bias", "mlp2.6.bias", "fuse_sem.0.bias",
               "per_point_out.0.bias")  # Conv->BN->ReLU only; Conv->ReLU->BN biases are real


def check_grad(got, ref, name, sd_grads, rel=3e-3):
    """Biases that feed a training-mode BatchNorm have an exactly-zero true gradient (BN
    subtracts the batch mean), so both sides hold only rounding noise: require that noise to be
    small against the layer's weight gradient instead of comparing noise to noise."""
    if name in BN_FED_BIAS:
        wg = sd_grads[name.replace(".bias", ".weight")].abs().max().item()
        assert got.abs().max().item() <= 1e-3 * max(wg, 1e-6), name
        return
    close(got, ref, rel, name + ".grad")


def _req(P):
    for k, v in P.items():
        if v.dtype.is_floating_point and "running" not in k:
            v.requires_grad_(True)


@pytest.mark.parametrize("n", [256, 96])
def test_target_encoder_fwd_bwd(dev, n):
    P, tgt, _, _ = _mods(dev)
    Pt = P["target_encoder_full"]
    _req(Pt)
    g = torch.Generator().manual_seed(n)
    x = torch.rand(2, n, 3, generator=g) * 2 - 1
    sem = torch.randn(2, n, 16, generator=g)
    w1, w2 = torch.randn(2, 64, generator=g), torch.randn(2, 64, n, generator=g)
    code, pp = tgt(x.to(dev), sem.to(dev))
    ((code * w1.to(dev)).sum() + (pp * w2.to(dev)).sum()).backward()
    rc, rpp = ured_ref.target_encoder(Pt, x, sem, False)
    ((rc * w1).sum() + (rpp * w2).sum()).backward()
    close(code, rc, 2e-4, "code")
    close(pp, rpp, 2e-4, "per_point")
    sd = dict(tgt.named_parameters())
    for k, v in Pt.items():
        if k.startswith("stn") or not v.dtype.is_floating_point:
            continue
        if "running" in k:
            close(dict(tgt.named_buffers())[k], v, 1e-4, k)
        else:
            check_grad(sd[k].grad, v.grad, k, {n: p.grad for n, p in sd.items()})
    assert int(tgt.mlp1[1].num_batches_tracked) == 1


@pytest.mark.parametrize("n", [128, 40])
def test_source_encoder_fwd_bwd(dev, n):
    P, _, src, _ = _mods(dev)
    Ps = P["src_encoder_all"]
    _req(Ps)
    g = torch.Generator().manual_seed(n + 1)
    x = torch.rand(2, 3, n, 3, generator=g) - 0.5
    sem = torch.randn(2, 3, 16, generator=g)
    w1, w2 = torch.randn(6, 64, generator=g), torch.randn(6, 64, n, generator=g)
    code, pp = src(x.to(dev), sem.to(dev))
    ((code * w1.to(dev)).sum() + (pp * w2.to(dev)).sum()).backward()
    rc, rpp = ured_ref.target_encoder(Ps, x, sem, True)
    ((rc * w1).sum() + (rpp * w2).sum()).backward()
    close(code, rc, 2e-4, "code")
    close(pp, rpp, 2e-4, "per_point")
    sd = dict(src.named_parameters())
    for k, v in Ps.items():
        if k.startswith("stn") or not v.dtype.is_floating_point or "running" in k:
            continue
        check_grad(sd[k].grad, v.grad, k, {n: p.grad for n, p in sd.items()})


def test_encoder_eval_mode(dev):
    P, tgt, _, _ = _mods(dev)
    Pt = P["target_encoder_full"]
    g = torch.Generator().manual_seed(9)
    x = torch.rand(2, 128, 3, generator=g)
    sem = torch.randn(2, 128, 16, generator=g)
    with torch.no_grad():
        tgt(x.to(dev), sem.to(dev))                      # one train step moves the running stats
        ured_ref.target_encoder(Pt, x, sem, False)
        tgt.eval()
        code, pp = tgt(x.to(dev), sem.to(dev))
        rc, rpp = ured_ref.target_encoder(Pt, x, sem, False, training=False)
    close(code, rc, 2e-4, "code_eval")
    close(pp, rpp, 2e-4, "pp_eval")


@pytest.mark.parametrize("code_first,ragged", [(False, False), (True, False), (False, True)])
def test_residual_net_split(dev, code_first, ragged):
    P, _, _, rn = _mods(dev)
    Pr = P["recon_decoder_full"]
    _req(Pr)
    g = torch.Generator().manual_seed(11)
    M, G = 600, 5
    pp = torch.randn(M, 64, generator=g, requires_grad=True)
    code = torch.randn(G, 64, generator=g, requires_grad=True)
    if ragged:
        cuts = torch.tensor([0, 100, 101, 350, 350, 600])
        gid = torch.repeat_interleave(torch.arange(G), cuts[1:] - cuts[:-1])
        kw = dict(gidx=gid.int().to(dev), off=cuts.int().to(dev))
    else:
        M = 600
        gid = torch.arange(M) // 120
        kw = dict(group_rows=120)
    feat = torch.cat([code[gid], pp], 1) if code_first else torch.cat([pp, code[gid]], 1)
    ref = ured_ref.residual_net(Pr, feat.unsqueeze(0)).squeeze(0)
    w = torch.randn(ref.shape, generator=g)
    (ref * w).sum().backward()
    ppd = pp.detach().to(dev).requires_grad_(True)
    cd = code.detach().to(dev).requires_grad_(True)
    out = rn.forward_split(ppd, cd, code_first=code_first, **kw)
    (out * w.to(dev)).sum().backward()
    close(out, ref, 2e-4, "out")
    close(ppd.grad, pp.grad, 2e-3, "dpp")
    close(cd.grad, code.grad, 2e-3, "dcode")
    sd = dict(rn.named_parameters())
    for k, v in Pr.items():
        if v.dtype.is_floating_point and "running" not in k:
            check_grad(sd[k].grad, v.grad, k, {n: p.grad for n, p in sd.items()})


def test_residual_net_plain_forward(dev):
    P, _, _, rn = _mods(dev)
    g = torch.Generator().manual_seed(12)
    f = torch.randn(2, 80, 128, generator=g)
    close(rn(f.to(dev)), ured_ref.residual_net(P["recon_decoder_full"], f), 2e-4, "plain")


@pytest.mark.parametrize("Cout,Kin,pro,M", [(3, 32, 0, 70001), (64, 3, 0, 4099), (3, 64, 1, 20000),
                                            (3, 128, 2, 513), (256, 4, 0, 255), (5, 3, 1, 1000),
                                            (2, 64, 0, 100), (64, 1, 1, 37), (4, 96, 2, 1), (3, 32, 0, 0)])
def test_wgrad_skinny_edge_layers(K, dev, Cout, Kin, pro, M):
    """The 3-channel edge layers' weight gradients (ured_wgrad_skinny): strided dY/X views,
    a column offset into X, the encoder prologues, accumulate into an existing gradient."""
    g = torch.Generator().manual_seed(Cout * 1000 + Kin + pro)
    ldd, ldx, xoff = Cout + 5, Kin + 7, 3
    if M % 2:                                   # also the aligned float4 path
        ldd, ldx, xoff = Cout, Kin, 0
    dY = torch.randn(M, ldd, generator=g)
    X = torch.randn(M, ldx, generator=g)
    s, t = torch.rand(Kin, generator=g) + 0.5, torch.randn(Kin, generator=g)
    prev = torch.randn(Cout, Kin, generator=g)
    x = X[:, xoff:xoff + Kin].double()
    h = {0: x, 1: torch.relu(x * s.double() + t.double()), 2: torch.relu(x) * s.double() + t.double()}[pro]
    ref = dY[:, :Cout].double().t() @ h
    out = torch.empty(Cout, Kin, device=dev)
    kw = dict(pro=pro, pro_s=s.to(dev), pro_t=t.to(dev)) if pro else {}
    K.wgrad(dY.to(dev), ldd, X.to(dev), ldx, Cout, Kin, M, out, Kin, X_off=xoff, **kw)
    close(out, ref, 1e-5, "wgrad skinny")
    acc = prev.to(dev)
    K.wgrad(dY.to(dev), ldd, X.to(dev), ldx, Cout, Kin, M, acc, Kin, X_off=xoff, accumulate=True, **kw)
    close(acc, ref + prev.double(), 1e-5, "wgrad skinny accumulate")


@pytest.mark.parametrize("M,N,Kd", [(32768, 1024, 1024), (8192, 512, 512), (4096, 256, 1152)])
def test_gemm_fp32_accuracy_vs_float64(dev, M, N, Kd):
    """The MLP GEMMs (v_mfma_f32_32x32x2_f32, csrc/mlp.hip gemm2_kernel) against float64 matmuls
    of the same fp32 inputs at step-like shapes: forward with the BN+ReLU prologue, dgrad with a
    k-major weight and split-K wgrad within 4e-6 of max |y| (measured 1.1e-6 to 1.6e-6,
    tools/emu_accuracy.py), and bitwise equal from run to run."""
    from ured_hip import kernels as K
    g = torch.Generator(device=dev).manual_seed(M + N)
    X = torch.randn(M, Kd, device=dev, generator=g)
    W = torch.randn(N, Kd, device=dev, generator=g) * Kd ** -0.5
    s = torch.rand(Kd, device=dev, generator=g) + 0.5
    t = torch.randn(Kd, device=dev, generator=g) * 0.1
    Y = torch.empty(M, N, device=dev)
    K.gemm(M, N, Kd, X, Kd, W, Kd, Y, N, pro_a=K.PRO_ENC, pro_s=s, pro_t=t)
    dY = torch.randn(M, N, device=dev, generator=g)
    G = torch.empty(M, Kd, device=dev)
    K.gemm(M, Kd, N, dY, N, W, Kd, G, Kd, b_kmajor=True)
    dW = torch.empty(N, Kd, device=dev)
    K.wgrad(dY, N, X, Kd, N, Kd, M, dW, Kd)
    refs = {"fwd": (Y, torch.relu(X.double() * s.double() + t.double()) @ W.double().t()),
            "dgrad": (G, dY.double() @ W.double()), "wgrad": (dW, dY.double().t() @ X.double())}
    for name, (y, r) in refs.items():
        e = float((y.double() - r).abs().max() / r.abs().max())
        assert e <= 4e-6, (name, e)
    Y2, G2, dW2 = torch.empty_like(Y), torch.empty_like(G), torch.empty_like(dW)     # run to run: bitwise
    K.gemm(M, N, Kd, X, Kd, W, Kd, Y2, N, pro_a=K.PRO_ENC, pro_s=s, pro_t=t)
    K.gemm(M, Kd, N, dY, N, W, Kd, G2, Kd, b_kmajor=True)
    K.wgrad(dY, N, X, Kd, N, Kd, M, dW2, Kd)
    assert torch.equal(Y, Y2) and torch.equal(G, G2) and torch.equal(dW, dW2)
