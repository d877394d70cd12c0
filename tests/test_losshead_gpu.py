"""The fused loss head (ured_hip/losshead.py, csrc/loss.hip) against the oracle's loss functions
in float64 (oracle/ured_ref.py: compute_cm_loss, residual_retrieval_loss, pc_consistency[_weighted],
contrast_loss — each pinned to the reference by tests/test_oracle_golden.py) on the same inputs,
and the whole train step with the head against the composed torch form.

Tolerances: loss terms 2e-6 relative (fp32 sums of up to 5e5 terms vs float64); gradients
elementwise within 1e-5 of the tensor's largest entry (the oracle's NN indices are the same
fp32 contract; the head only reorders fp32 sums).
"""
import numpy as np
import pytest
import torch

import step_parity
from oracle import ured_ref

pytestmark = pytest.mark.gpu

W = {"use_chamfer_loss": 30.0, "use_chamfer_part_loss": 1.0, "use_symmetry_loss": 30.0, "use_contrast_loss": 0.5,
     "use_param_loss": 0.0, "init_p_m_loss": -1, "use_residuals_reg": 3.0, "use_recon": 30.0}


def _inputs(dev, B, N, parts, C=32, NP=64, P=16, U=None, seed=0, dup=True):
    from ured_hip.ops import build_parts
    g = torch.Generator().manual_seed(seed)
    S = P * NP
    x = torch.rand(B, N, 3, generator=g) * 2 - 1
    labels = torch.stack([torch.sort(torch.randint(0, k, (N,), generator=g)).values for k in parts])
    for b, k in enumerate(parts):           # every label present
        labels[b, :k] = torch.arange(k)
    labels = torch.sort(labels, dim=1).values
    perm = torch.stack([torch.randperm(N, generator=g) for _ in range(B)])   # points not grouped by part
    labels = torch.gather(labels, 1, perm)
    out = torch.rand(B, S, 3, generator=g) * 2 - 1
    res = torch.randn(B, N, 3, generator=g) * 0.1
    rec = torch.randn(B, N, 3, generator=g) * 0.5
    src_labels = torch.full((B, P), -1, dtype=torch.long)
    for b, k in enumerate(parts):
        src_labels[b, :k] = torch.randint(0, 50, (k,), generator=g)
    if not dup:
        src_labels[0, 0] = -1              # an ignored contrast row among the valid parts
    U = U or B * P
    inv = torch.randint(0, U, (B * P,), generator=g) if dup else torch.arange(B * P) % U
    recu = torch.randn(U, NP, 3, generator=g) * 0.3
    ptsu = torch.randn(U, NP, 3, generator=g) * 0.3
    t = torch.randn(B, P, C, generator=g)
    s = torch.randn(B, P, C, generator=g)
    parts_d = build_parts(labels.to(dev), x.to(dev), P)
    return dict(x=x, labels=labels, out=out, res=res, rec=rec, src_labels=src_labels, inv=inv, recu=recu, ptsu=ptsu,
                t=t, s=s, parts=parts_d, NP=NP, P=P)


def _oracle(d, cfg):
    """float64 oracle terms and gradients (out, res, rec, recu, t, s)."""
    B, P, NP = d["x"].shape[0], d["P"], d["NP"]
    X = d["x"].double()
    lab = d["labels"]
    part_x = [[X[b, lab[b] == v] for v in torch.unique(lab[b])] for b in range(B)]
    k = torch.tensor([len(p) for p in part_x])
    mask = (torch.arange(P).unsqueeze(0) < k.unsqueeze(1)).double()
    leaves = {n: d[n].double().requires_grad_(True) for n in ("out", "res", "rec", "recu", "t", "s")}
    out = leaves["out"]
    T = {}
    T["cd_loss_full"], T["cd_loss_part"] = ured_ref.compute_cm_loss(out, X, part_x, mask, np_per_part=NP)
    T["ref_cd_loss_full"], T["ref_cd_loss_part"] = ured_ref.compute_cm_loss(ured_ref.get_symmetric(out), X, part_x,
                                                                            mask, np_per_part=NP)
    T["re_reg_loss_full"], T["reg_loss_full"] = ured_ref.residual_retrieval_loss(X, out.detach(), leaves["res"], mask,
                                                                                 np_per_part=NP)
    T["recon_loss_full"] = ured_ref.pc_consistency(leaves["rec"], X)
    inv = d["inv"]
    T["recon_loss_src"] = ured_ref.pc_consistency_weighted(leaves["recu"][inv].view(B, P, NP, 3),
                                                           d["ptsu"].double()[inv].view(B, P, NP, 3), mask)
    sl = d["src_labels"]
    T["contrast_loss"] = ured_ref.contrast_loss(leaves["t"], leaves["s"], torch.where(sl >= 0, 1, sl))
    loss = (T["cd_loss_full"] * cfg["use_chamfer_loss"] + T["cd_loss_part"] * cfg["use_chamfer_part_loss"]
            + T["contrast_loss"] * cfg["use_contrast_loss"] + T["ref_cd_loss_full"] * cfg["use_symmetry_loss"]
            + T["re_reg_loss_full"] * cfg["use_residuals_reg"] + T["reg_loss_full"] * cfg["use_residuals_reg"] * 0.01
            + T["recon_loss_full"] * cfg["use_recon"] + T["recon_loss_src"] * cfg["use_recon"])
    loss.backward()
    T["all_loss"] = loss
    return {k: float(v) for k, v in T.items()}, {n: v.grad for n, v in leaves.items()}


@pytest.mark.parametrize("B,N,parts,dup", [(2, 200, (3, 5), True), (3, 130, (1, 16, 7), False),
                                           (4, 96, (2, 2, 4, 9), True)])
def test_loss_head_matches_oracle(dev, B, N, parts, dup):
    from ured_hip.losshead import HeadInputs, loss_head
    d = _inputs(dev, B, N, parts, dup=dup)
    leaves = {n: d[n].to(dev).requires_grad_(True) for n in ("out", "res", "rec", "recu", "t", "s")}
    hi = HeadInputs(d["x"].to(dev), d["parts"], d["NP"], d["src_labels"].to(dev), d["ptsu"].to(dev),
                    d["inv"].to(dev), W, gate=True)
    loss, T, knn = loss_head(hi, leaves["out"], leaves["res"], leaves["rec"], leaves["recu"], leaves["t"], leaves["s"])
    loss.backward()
    rT, rG = _oracle(d, W)
    got = {k: float(v) for k, v in T.items()}
    got["all_loss"] = float(loss)
    for k in rT:
        assert abs(got[k] - rT[k]) <= 2e-6 * abs(rT[k]), (k, got[k], rT[k])
    for n, r in rG.items():
        g = leaves[n].grad.double().cpu()
        dev_ = (g - r).abs().max().item() / max(r.abs().max().item(), 1e-30)
        assert dev_ <= 1e-5, f"d{n}: {dev_:.2e}"
    # the knn output is the x -> out NN index of every target point (first half)
    from oracle import nn_ref
    for b in range(B):
        kb = len(set(d["labels"][b].tolist()))
        _, ri = nn_ref.nn_dir(d["x"][b].numpy(), d["out"][b, :kb * d["NP"]].numpy())
        np.testing.assert_array_equal(knn[b].cpu().numpy(), ri)


def test_loss_head_param_and_external_contrast(dev):
    """use_param_loss: the external param term is added first (engine/train.py:281-283) and gets
    w * g back; contrast_ext (the multi-rank path) replaces the fused contrastive loss."""
    from ured_hip.losshead import HeadInputs, loss_head
    d = _inputs(dev, 2, 150, (4, 3))
    cfg = dict(W, use_param_loss=2.0)
    mk = lambda: {n: d[n].to(dev).requires_grad_(True) for n in ("out", "res", "rec", "recu", "t", "s")}   # noqa: E731
    hi = HeadInputs(d["x"].to(dev), d["parts"], d["NP"], d["src_labels"].to(dev), d["ptsu"].to(dev),
                    d["inv"].to(dev), cfg, gate=True)
    a = mk()
    param = torch.tensor(0.75, device=dev, requires_grad=True)
    con = torch.tensor(1.25, device=dev, requires_grad=True)
    loss, T, _ = loss_head(hi, a["out"], a["res"], a["rec"], a["recu"], a["t"], a["s"], param, con)
    loss.backward()
    b = mk()
    hi0 = HeadInputs(d["x"].to(dev), d["parts"], d["NP"], d["src_labels"].to(dev), d["ptsu"].to(dev),
                     d["inv"].to(dev), W, gate=True)
    loss0, T0, _ = loss_head(hi0, b["out"], b["res"], b["rec"], b["recu"], b["t"], b["s"])
    exp = 0.75 * 2.0 + (float(loss0) - float(T0["contrast_loss"]) * 0.5) + 1.25 * 0.5
    assert abs(float(loss) - exp) <= 1e-5 * abs(exp)
    assert float(T["param_loss"]) == 0.75 and float(T["contrast_loss"]) == 1.25
    assert float(param.grad) == 2.0 and float(con.grad) == 0.5
    assert a["t"].grad is None and a["s"].grad is None     # the contrastive gradient went to con


def test_loss_head_gate_off_drops_residual_terms(dev):
    """epoch <= init_p_m_loss: the residual terms are not in the loss (engine/train.py:308) and the
    residual net gets NO gradient from the head (None, so Adam skips it, as torch does)."""
    from ured_hip.losshead import HeadInputs, loss_head
    d = _inputs(dev, 2, 120, (2, 3))
    hi = HeadInputs(d["x"].to(dev), d["parts"], d["NP"], d["src_labels"].to(dev), d["ptsu"].to(dev),
                    d["inv"].to(dev), W, gate=False)
    a = {n: d[n].to(dev).requires_grad_(True) for n in ("out", "res", "rec", "recu", "t", "s")}
    loss, T, _ = loss_head(hi, a["out"], a["res"], a["rec"], a["recu"], a["t"], a["s"])
    loss.backward()
    assert "re_reg_loss_full" not in T and "reg_loss_full" not in T
    assert a["res"].grad is None and a["out"].grad is not None


@pytest.mark.parametrize("unique", [True, False], ids=["unique_sources", "all_slots"])
def test_step_head_matches_composed(dev, unique):
    """The train step with the loss head == the composed torch form (same kernels elsewhere):
    every loss term within 2e-6 relative, every gradient tensor within 1e-4 (norm) / 1e-3
    (elementwise) of the composed step's — two fp32 orders of the same sums."""
    from test_train_step_gpu import _setup, TERMS
    ts1, b1, P, ob, cfg = _setup(dev, N=256, parts=(5, 2), unique=unique)
    ts2, b2, _, _, _ = _setup(dev, N=256, parts=(5, 2), unique=unique, loss_head=False)
    assert ts1.loss_head and not ts2.loss_head
    l1, T1 = ts1.forward(b1)
    l2, T2 = ts2.forward(b2)
    for k in TERMS:
        a, b = T1[k].item(), T2[k].item()
        assert abs(a - b) <= 2e-6 * abs(b), (k, a, b)
    l1.backward()
    l2.backward()
    ref = {(m, k): (None if p.grad is None else p.grad.detach().double().cpu())
           for m in step_parity.TRAINED for k, p in ts2.models[m].named_parameters()}
    step_parity.check_grads(ts1.models, ref, "head vs composed", grad_rel=1e-4, grad_elem=1e-3)
