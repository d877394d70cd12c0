"""The whole U-RED training step on the HIP path vs the CPU oracle (same weights, same batch).

The oracle runs in float64 (weights and inputs; its chamfer primitive stays the fp32 contract
formula). Tolerances (tests/step_parity.py): every loss term 1e-5 relative, every
parameter gradient tensor compared whole — relative norm of the difference and elementwise max
deviation — with the exactly-zero true gradients (BN-fed conv biases, attention key biases) at
noise level; deformed shape 1e-4 relative.
"""
import numpy as np
import pytest
import torch

import step_parity
from oracle import ured_ref

pytestmark = pytest.mark.gpu

CFG = {"source_latent_dim": 64, "target_latent_dim": 64, "sem_latent_dim": 16, "MAX_NUM_PARTS": 16,
       "alpha": 0.1, "use_chamfer_loss": 30.0, "use_chamfer_part_loss": 1.0, "use_symmetry_loss": 30.0,
       "use_contrast_loss": 0.5, "use_param_loss": 0.0, "init_p_m_loss": -1, "use_residuals_reg": 3.0,
       "use_recon": 30.0, "batch_size": 2, "device": "cuda", "optimizer": "adam", "learning_rate": 1e-3,
       "weight_decay": 5e-4, "lr_stepsize": 3, "lr_decay": 0.5, "momentum": 0.9}


def _setup(dev, B=2, N=128, parts=(3, 2), ns=24, seed=4, unique=True, **over):
    from dataset import synthetic
    from train_utils.load_sources import SourceDB
    from engine.train import TrainStep, batch_to_device
    db_np = synthetic.make_source_db(ns, seed=3)
    bt = synthetic.make_batch(B, N, ns, max_parts=16, parts=list(parts), seed=seed)
    db = SourceDB(db_np["src_points"], db_np["src_mats"], db_np["src_default_param"], db_np["src_sem"], dev)
    cfg = dict(CFG, batch_size=B, **over)
    ts = TrainStep(cfg, db, dev)
    P = ured_ref.make_params(cfg, seed=7)
    for name, sd in P.items():
        ts.models[name].load_state_dict(sd, strict=True)
    batch = batch_to_device(bt, dev, ns if unique else None)
    ob = {"src_points": torch.from_numpy(db_np["src_points"]), "src_mats": torch.from_numpy(db_np["src_mats"]),
          "src_sem": torch.from_numpy(db_np["src_sem"]), "src_index": torch.from_numpy(bt["src_index"]),
          "tgt_sem": torch.from_numpy(bt["tgt_sem"]), "x": torch.from_numpy(bt["x"]),
          "labels": torch.from_numpy(bt["labels"]).float(), "src_labels": torch.from_numpy(bt["src_labels"])}
    ob["src_labels"] = torch.where(ob["src_labels"] >= 0, torch.ones_like(ob["src_labels"]), ob["src_labels"])
    # the oracle runs in float64: early-layer gradient norms of an fp32 CPU run carry ~2e-3 of
    # rounding noise at these sizes (measured), more than the HIP path (fp64 BN statistics)
    for mod in P.values():
        for k in list(mod):
            if mod[k].dtype.is_floating_point:
                mod[k] = mod[k].double()
                if "running" not in k:
                    mod[k].requires_grad_(True)
    for k in ("src_points", "src_mats", "x", "labels"):
        ob[k] = ob[k].double()
    return ts, batch, P, ob, cfg


BN_FED_BIAS = ("mlp1.0.bias", "mlp1.3.bias", "mlp2.0.bias", "mlp2.3.bias", "mlp2.6.bias", "fuse_sem.0.bias",
               "per_point_out.0.bias", "fc.0.bias")

TERMS = ("cd_loss_full", "cd_loss_part", "contrast_loss", "ref_cd_loss_full", "ref_cd_loss_part",
         "re_reg_loss_full", "reg_loss_full", "recon_loss_full", "recon_loss_src", "all_loss")


def _oracle_grads(P):
    return {(mod, k): (None if v.grad is None else v.grad.detach().clone())
            for mod, sd in P.items() if mod != "embedding_layer"
            for k, v in sd.items() if torch.is_tensor(v) and v.requires_grad}


def _oracle_grads32(P, ob, cfg):
    """The same oracle step in fp32: the per-tensor fp32 noise floor (tests/step_parity.py)."""
    P32 = {m: {k: (v.detach().float().requires_grad_(True) if v.dtype.is_floating_point and "running" not in k
                   else v.detach().float() if v.dtype.is_floating_point else v.detach().clone())
               for k, v in sd.items()} for m, sd in P.items()}
    ob32 = {k: (v.float() if v.dtype.is_floating_point else v) for k, v in ob.items()
            if not k.startswith("_")}          # its own discrete choices: the fp32 noise floor
    loss, _ = ured_ref.train_forward(P32, ob32, cfg)
    loss.backward()
    return _oracle_grads(P32)


@pytest.mark.parametrize("unique", [True, False], ids=["unique_sources", "all_slots"])
@pytest.mark.parametrize("N,parts", [(128, (3, 2)), (512, (4, 4)), (256, (16, 1))])
def test_train_step_matches_oracle(dev, N, parts, unique):
    """unique: the source encoder / recon_decoder_src run once per distinct source part with
    row multiplicities (the oracle always encodes every slot, as the reference does). Every loss
    term within 1e-5 relative and every gradient tensor elementwise (tests/step_parity.py)."""
    ts, batch, P, ob, cfg = _setup(dev, N=N, parts=parts, unique=unique)
    if unique:
        assert batch["src_unique"].U < 2 * 16   # padding slots collapse onto one source part
    step_parity.record_pools(ts.models)
    loss, T = ts.forward(batch)
    # the oracle routes each pooled gradient to the point the HIP step chose (checked to be a
    # max up to fp32 noise: near-ties may resolve either way under a different summation order)
    ob["_pool_idx"] = step_parity.gpu_pool_choices(ts.models, batch, unique)
    ob["_pool_gpu"] = step_parity.gpu_pool_values(ts.models, batch, unique)
    ob["_nn_out"] = T["_out"].detach().cpu()      # NN indices: the HIP step's near-tie choices too
    ured_ref.NN_TIE_STATS.clear()
    rloss, R = ured_ref.train_forward(P, ob, cfg)
    label = f"N={N} parts={parts} unique={unique}"
    step_parity.tie_report(R["_pool"], label)
    step_parity.check_loss_terms({k: T[k].item() for k in TERMS}, {k: R[k].item() for k in TERMS}, label)
    o, ro = T["_out"].detach().cpu(), R["_out"].detach()
    assert (o - ro).abs().max().item() <= 1e-4 * ro.abs().max().item()
    loss.backward()
    rloss.backward()
    n, _ = step_parity.check_grads(ts.models, _oracle_grads(P), label, ref32=_oracle_grads32(P, ob, cfg))
    assert n >= 145


@pytest.mark.parametrize("case", ["param_loss", "complementme", "both"])
def test_train_step_param_loss_complementme(dev, case):
    """The two reference keys off in the shipped config (engine/train.py:192-194, 281-283):
    use_param_loss > 0 adds regularization_param(params_full, mask_part) (a new loss term, and
    gradient into the DeformNet through it); complementme z-flips the targets. Both vs the
    oracle, loss terms and every gradient tensor."""
    over = {"param_loss": {"use_param_loss": 1.0}, "complementme": {"complementme": True},
            "both": {"use_param_loss": 0.5, "complementme": True}}[case]
    ts, batch, P, ob, cfg = _setup(dev, N=256, parts=(4, 2), **over)
    step_parity.record_pools(ts.models)
    loss, T = ts.forward(batch)
    ob["_pool_idx"] = step_parity.gpu_pool_choices(ts.models, batch, True)
    ob["_pool_gpu"] = step_parity.gpu_pool_values(ts.models, batch, True)
    ob["_nn_out"] = T["_out"].detach().cpu()
    ured_ref.NN_TIE_STATS.clear()
    rloss, R = ured_ref.train_forward(P, ob, cfg)
    step_parity.tie_report(R["_pool"], case)
    terms = TERMS + (("param_loss",) if "use_param_loss" in over else ())
    assert ("param_loss" in T) == ("use_param_loss" in over)
    step_parity.check_loss_terms({k: T[k].item() for k in terms}, {k: R[k].item() for k in terms}, case)
    loss.backward()
    rloss.backward()
    step_parity.check_grads(ts.models, _oracle_grads(P), case, ref32=_oracle_grads32(P, ob, cfg))
    if "complementme" in over:      # the flip really happened: the un-flipped step differs
        ts2, batch2, _, _, _ = _setup(dev, N=256, parts=(4, 2))
        _, T2 = ts2.forward(batch2)
        assert abs(T2["recon_loss_full"].item() - T["recon_loss_full"].item()) > 1e-6


def test_train_step_runs_and_updates(dev):
    ts, batch, P, ob, cfg = _setup(dev)
    w0 = ts.models["param_decoder_full"].param_decoder[2].weight.detach().clone()
    T1 = ts.step(batch)
    T2 = ts.step(batch)
    assert torch.isfinite(T1["all_loss"]) and torch.isfinite(T2["all_loss"])
    assert not torch.equal(w0, ts.models["param_decoder_full"].param_decoder[2].weight.detach())
    assert int(ts.models["target_encoder_full"].mlp1[1].num_batches_tracked) == 2


def test_unique_sources_equal_all_slots(dev):
    """Unique-source encoding vs encoding all B x 16 slots on the GPU: same losses, gradients
    and BN running statistics up to fp32 summation order."""
    from engine.train import batch_to_device
    ts1, b1, P, ob, cfg = _setup(dev, N=256, parts=(5, 2), unique=True)
    ts2, b2, _, _, _ = _setup(dev, N=256, parts=(5, 2), unique=False)
    assert "src_unique" in b1 and "src_unique" not in b2
    l1, T1 = ts1.forward(b1)
    l2, T2 = ts2.forward(b2)
    for k in TERMS:
        a, b = T1[k].item(), T2[k].item()
        assert abs(a - b) <= 1e-5 * abs(b) + 1e-7, f"{k}: {a} vs {b}"
    l1.backward()
    l2.backward()
    for name in ("src_encoder_all", "recon_decoder_src"):
        m1, m2 = ts1.models[name], ts2.models[name]
        p2 = dict(m2.named_parameters())
        for k, p in m1.named_parameters():
            if p.grad is None:
                assert p2[k].grad is None
                continue
            if k in BN_FED_BIAS:
                continue
            d = (p.grad - p2[k].grad).norm().item()
            assert d <= 2e-3 * p2[k].grad.norm().item() + 1e-5, f"{name}.{k}: |diff| {d}"
        b2s = dict(m2.named_buffers())
        for k, v in m1.named_buffers():
            if v.dtype.is_floating_point:
                assert torch.allclose(v, b2s[k], rtol=1e-4, atol=1e-6), f"{name}.{k}"
            else:
                assert torch.equal(v, b2s[k])


@pytest.mark.parametrize("flat", [True, False], ids=["flat_adam", "torch_adam"])
def test_fused_clip_matches_clip_grad_norm(dev, flat):
    """TrainStep.clip_and_step's clipping == torch.nn.utils.clip_grad_norm_ per module
    (engine/train.py:331-336) up to fp32 rounding of the six module norms: the one-launch norm
    path before torch's Adam, and FlatAdam's fused tail (the gradients it leaves are the clipped
    ones)."""
    from engine.train import CLIPPED
    ts = _setup(dev, flat_adam=flat)[0]
    assert (type(ts.optimizer).__name__ == "FlatAdam") == flat
    for name in CLIPPED:                      # large gradients so that every module is clipped
        for p in ts.models[name].parameters():
            p.grad = torch.randn_like(p) * 10.0
    ref = {name: [p.grad.clone() for p in ts.models[name].parameters()] for name in CLIPPED}
    for name in CLIPPED:
        gs = ref[name]                        # clip_grad_norm_'s arithmetic on the copies
        total = torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(g) for g in gs]))
        coef = (5.0 / (total + 1e-6)).clamp(max=1.0)
        for g in gs:
            g.mul_(coef)
    if not flat:
        ts.optimizer.step = lambda: None      # clip only
    ts.clip_and_step()
    for name in CLIPPED:
        for p, r in zip(ts.models[name].parameters(), ref[name]):
            torch.testing.assert_close(p.grad, r, rtol=2e-6, atol=1e-9)


def test_flat_adam_matches_torch_adam(dev):
    """FlatAdam (flat buffers, ured_adam_clip_step) == torch.optim.Adam(fused=True) with the same
    L2 weight decay over several steps, gradients present on only some parameters (the others
    untouched, as torch skips them), an lr change in between (StepLR's path), no clipping."""
    from ured_hip.optim import FlatAdam
    g = torch.Generator().manual_seed(3)
    shapes = [(64, 3), (64,), (128, 64), (5,), (1024, 33), (7, 7)]
    base = [torch.randn(*s, generator=g) for s in shapes]
    pa = [torch.nn.Parameter(b.clone().to(dev)) for b in base]
    pb = [torch.nn.Parameter(b.clone().to(dev)) for b in base]
    fa = FlatAdam(pa, [pa[:3], pa[3:]], lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=5e-4)
    ta = torch.optim.Adam(pb, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=5e-4, fused=True)
    live = [0, 1, 2, 4, 5]                    # parameter 3 never gets a gradient
    for it in range(5):
        if it == 3:
            for o in (fa, ta):
                o.param_groups[0]["lr"] = 5e-4
        fa.zero_grad()
        ta.zero_grad()
        for i in live:
            gr = torch.randn(*shapes[i], generator=g).to(dev)
            pa[i].grad = gr.clone()
            pb[i].grad = gr.clone()
        fa.step()
        ta.step()
        for i in range(len(shapes)):
            torch.testing.assert_close(pa[i].detach(), pb[i].detach(), rtol=1e-6, atol=1e-7, msg=f"step {it} p{i}")
    assert torch.equal(pa[3].detach().cpu(), base[3])
    assert fa.flat_grad is not None and pa[0].data_ptr() == fa.flat_param.data_ptr()


def test_flat_adam_parameter_set_changes(dev):
    """Parameters whose gradient appears later (p2 from step 2: the residual net once
    epoch > init_p_m_loss) or disappears (p4 after step 2) follow torch's Adam exactly: no update
    while they have no gradient (no weight decay, no moment decay) and a per-parameter step count
    (bias corrections restart from 1 for a parameter that joins late)."""
    from ured_hip.optim import FlatAdam
    g = torch.Generator().manual_seed(5)
    shapes = [(64, 3), (64,), (128, 64), (5,), (1024, 33), (7, 7)]
    base = [torch.randn(*s, generator=g) for s in shapes]
    pa = [torch.nn.Parameter(b.clone().to(dev)) for b in base]
    pb = [torch.nn.Parameter(b.clone().to(dev)) for b in base]
    fa = FlatAdam(pa, [pa[:3], pa[3:]], lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=5e-4)
    ta = torch.optim.Adam(pb, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=5e-4, fused=True)
    for it in range(6):
        live = [0, 1, 3, 5] + ([2] if it >= 2 else []) + ([4] if it < 2 else [])
        fa.zero_grad()
        ta.zero_grad()
        for i in live:
            gr = torch.randn(*shapes[i], generator=g).to(dev)
            pa[i].grad = gr.clone()
            pb[i].grad = gr.clone()
        fa.step(max_norm=0.0)
        ta.step()
        for i in range(len(shapes)):
            torch.testing.assert_close(pa[i].detach(), pb[i].detach(), rtol=1e-6, atol=1e-7, msg=f"step {it} p{i}")
        for i in range(len(shapes)):
            assert (pa[i].grad is None) == (i not in live), (it, i)


def test_residual_net_joins_after_init_p_m_loss(dev):
    """init_p_m_loss = 0: the residual loss (and so re_residual_net_full's gradient) is off at
    epoch 0 and on from epoch 1 (engine/train.py:306-316). FlatAdam must leave the residual net
    untouched (bitwise) at epoch 0, and at epoch 1 take torch Adam's FIRST step for it (its own
    step count starts at 1: update = lr * g'/(|g'| + eps), g' = clipped g + wd * p), while the
    other modules take their third."""
    ts, batch = _setup(dev, flat_adam=True, init_p_m_loss=0)[:2]
    res = ts.models["re_residual_net_full"]
    res0 = {k: p.detach().clone() for k, p in res.named_parameters()}
    for ep in (0, 0):
        ts.step(batch, epoch=ep)
    for k, p in res.named_parameters():
        assert torch.equal(p.detach(), res0[k]), k
    T = ts.step(batch, epoch=1)
    assert "re_reg_loss_full" in T
    lr, eps, wd = 1e-3, 1e-8, 5e-4
    moved = 0
    for k, p in res.named_parameters():
        g = p.grad.detach().double()                      # the clipped gradient FlatAdam used
        gw = g + wd * res0[k].double()
        m, v = 0.1 * gw, 0.001 * gw * gw                  # first step: (1 - b1) g', (1 - b2) g'^2
        upd = (lr / 0.1) * m / (v.sqrt() / 0.001 ** 0.5 + eps)
        exp = res0[k].double() - upd
        torch.testing.assert_close(p.detach().double(), exp, rtol=0, atol=2e-7, msg=k)
        moved += int((p.detach() != res0[k]).sum())
    assert moved > 1000
    assert int(ts.optimizer.state["flat"]["step"].max()) == 3


def test_flat_adam_train_steps_match_torch_adam(dev):
    """Full training steps with FlatAdam vs torch's Adam + the one-launch clip. After one step
    the parameters agree to 1e-3 of the step's largest move (the clip factors differ in the last
    bit: fp64 vs per-tensor fp32 norm sums; Adam's update is scale-free); the losses agree to
    1e-5 over two steps; the third is only a gross check (1e-3): from there the runs drift apart
    chaotically (Adam's normalised update turns last-bit gradient differences of the BN-fed
    biases, exactly zero in exact arithmetic, into +-lr moves)."""
    ts1, batch = _setup(dev, flat_adam=True)[:2]
    ts2 = _setup(dev, flat_adam=False)[0]
    init = {name: {k: p.detach().clone() for k, p in m.named_parameters()} for name, m in ts2.models.items()}
    for it in range(3):
        T1, T2 = ts1.step(batch), ts2.step(batch)
        a, b = T1["all_loss"].item(), T2["all_loss"].item()
        # step 0: same parameters; later steps: the BN-fed biases' Adam noise (+-lr moves of an
        # exactly-zero true gradient) differs between the two clip arithmetics and grows
        assert abs(a - b) <= (1e-5 if it < 2 else 1e-3) * abs(b) + 1e-7, (it, a, b)
        if it > 0:
            continue
        for name, m in ts1.models.items():
            p2 = dict(ts2.models[name].named_parameters())
            move = max((p2[k].detach() - init[name][k]).abs().max().item() for k in p2)
            for k, p in m.named_parameters():
                if k in BN_FED_BIAS:
                    continue      # exactly-zero true gradient: Adam's update of the noise is +-lr either way
                d = (p.detach() - p2[k].detach()).abs().max().item()
                assert d <= 1e-3 * move + 1e-9, (name, k, d, move)


def test_bn_counters_count_steps(dev):
    """num_batches_tracked of every BatchNorm the HIP chain runs advances by one per training
    forward (the increment is folded into the statistics-finalize launch)."""
    ts, batch = _setup(dev)[:2]
    bns = [(n, m) for name in ("src_encoder_all", "target_encoder_full", "re_residual_net_full")
           for n, m in ts.models[name].named_modules() if isinstance(m, torch.nn.BatchNorm1d)]
    before = {n: int(m.num_batches_tracked) for n, m in bns}
    ts.step(batch)
    ts.step(batch)
    for n, m in bns:
        used = int(m.num_batches_tracked) - before[n]
        assert used in (0, 2), (n, used)      # 0: the module's unused stn1/stn2 branches
    assert sum(int(m.num_batches_tracked) - before[n] for n, m in bns) > 0
