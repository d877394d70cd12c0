"""Parity at the BASELINE configurations' stated sizes.

config 2  the training step at its real shape: bs=16, 2048 points, 16 x 1024 source slots,
          C=512, S=128, 512 sources (config/config_train_test.json), k=4 parts (12 of 16
          slots are padding copies of source[-1]) and k=16 (no padding), with unique-source
          encoding and with every slot encoded
config 3  retrieval + deformation inference (engine/test.py, vis.py semantics): bs=16, 2048
          points, C=512, 512 sources
config 5  a 4096-point training step (bs=8 per GPU: the per-rank share of global bs 64 over 8
          GPUs) and the NN kernel at 64 x 4096 x 4096

Oracle: oracle/ured_ref.py in float64 on the host (weights and inputs; its chamfer primitive is
the fp32 C contract of oracle/nn_oracle.c), ~30-50 s per configuration on 16 threads; one
oracle run serves both source-encoding modes of a configuration.

Tolerances (tests/step_parity.py, same rules as tests/test_train_step_gpu.py):
  * every loss term within 1e-5 relative; the deviations are printed;
  * the deformed shape within 1e-4 of its largest coordinate;
  * every parameter gradient tensor compared whole: ||g - g_ref|| / ||g_ref|| <= 1e-3 and the
    elementwise max deviation within 2e-3 of the tensor's largest entry, or 3x the deviation of
    the same oracle run in fp32 where fp32 accumulation alone moves a tensor further; the
    exactly-zero true gradients (BN-fed conv biases, attention key biases) at noise level;
  * NN distances and indices of the step's own chamfer families bit-exact against the C oracle
    run on the same (GPU-produced) inputs and segment tables;
  * retrieval indices bit-exact except where the oracle's top-2 cosine gap is < 1e-6 (SURVEY
    §8(d)); the near-tie count is printed.
"""
import json
import os

import numpy as np
import pytest
import torch

import step_parity
from conftest import PKG_DIR
from oracle import nn_ref, ured_ref

pytestmark = pytest.mark.gpu

TERMS = ("cd_loss_full", "cd_loss_part", "contrast_loss", "ref_cd_loss_full", "ref_cd_loss_part",
         "re_reg_loss_full", "reg_loss_full", "recon_loss_full", "recon_loss_src", "all_loss")
NS = 512
_ORACLE = {}


def _threads():
    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))


def _cfg(**over):
    with open(os.path.join(PKG_DIR, "config", "config_train_test.json")) as f:
        cfg = json.load(f)
    cfg.update(device="cuda", log_every=0)
    cfg.update(over)
    return cfg


def _params64(cfg, seed):
    P = ured_ref.make_params(cfg, seed=seed)
    P64 = {}
    for name, sd in P.items():
        d = {}
        for k, v in sd.items():
            if v.dtype.is_floating_point:
                v = v.double()
                if "running" not in k:
                    v.requires_grad_(True)
            d[k] = v
        P64[name] = d
    return P, P64


def _oracle_batch(db_np, bt, dtype=torch.float64):
    ob = {"src_points": torch.from_numpy(db_np["src_points"]).to(dtype),
          "src_mats": torch.from_numpy(db_np["src_mats"]).to(dtype),
          "src_sem": torch.from_numpy(db_np["src_sem"]), "src_index": torch.from_numpy(bt["src_index"]),
          "tgt_sem": torch.from_numpy(bt["tgt_sem"]), "x": torch.from_numpy(bt["x"]).to(dtype),
          "labels": torch.from_numpy(bt["labels"]).to(dtype)}
    sl = torch.from_numpy(bt["src_labels"])
    ob["src_labels"] = torch.where(sl >= 0, torch.ones_like(sl), sl)
    return ob


def _grads_of(P):
    return {(mod, k): (None if v.grad is None else v.grad.detach().clone())
            for mod, sd in P.items() if mod != "embedding_layer"
            for k, v in sd.items() if torch.is_tensor(v) and v.requires_grad}


def _oracle_floor(key, cfg, db_np, bt):
    """The oracle's gradients from an fp32 run (its own max-pool / NN choices), cached per
    configuration: the per-tensor fp32 noise floor of tests/step_parity.py."""
    if key not in _ORACLE:
        _threads()
        P, _ = _params64(cfg, seed=7)
        P32 = {m: {k: (v.clone().requires_grad_(True) if v.dtype.is_floating_point and "running" not in k else v.clone())
                   for k, v in sd.items()} for m, sd in P.items()}
        loss, R = ured_ref.train_forward(P32, _oracle_batch(db_np, bt, torch.float32), cfg)
        loss.backward()
        _ORACLE[key] = _grads_of(P32)
        del loss, R, P32
    return _ORACLE[key]


def _oracle64(cfg, db_np, bt, pool_idx=None, nn_out=None, pool_vals=None):
    """float64 oracle forward + backward -> (terms, out, gradients, its max-pool record).
    pool_idx / nn_out: the HIP step's max-pool winners and deformed shape, whose discrete choices
    (max-pool winners, NN indices) the oracle follows where they are near-ties of its own
    (ured_ref.max_pool, ured_ref._OracleNN: each checked, a non-tie raises)."""
    _threads()
    _, P64 = _params64(cfg, seed=7)
    ob = _oracle_batch(db_np, bt)
    if pool_idx is not None:
        ob["_pool_idx"] = pool_idx
        ob["_pool_gpu"] = pool_vals
    if nn_out is not None:
        ob["_nn_out"] = nn_out
    ured_ref.NN_TIE_STATS.clear()
    loss, R = ured_ref.train_forward(P64, ob, cfg)
    loss.backward()
    res = ({k: float(R[k]) for k in TERMS}, R["_out"].detach().float(), _grads_of(P64), R["_pool"])
    del loss, R, P64
    return res


def _run_step(dev, B, N, parts, unique, data_seed=4):
    from dataset import synthetic
    from engine.train import TrainStep, batch_to_device
    from train_utils.load_sources import SourceDB
    cfg = _cfg(batch_size=B, num_points=N, parts=parts)
    db_np = synthetic.make_source_db(NS, seed=3)
    bt = synthetic.make_batch(B, N, NS, parts=parts, seed=data_seed)
    db = SourceDB(db_np["src_points"], db_np["src_mats"], db_np["src_default_param"], db_np["src_sem"], dev)
    cfg["unique_sources"] = unique
    ts = TrainStep(cfg, db, dev)
    P, _ = _params64(cfg, seed=7)
    for name, sd in P.items():
        ts.models[name].load_state_dict(sd, strict=True)
    batch = batch_to_device(bt, dev, NS if unique else None)
    return cfg, db_np, bt, ts, batch


def _check_step(dev, B, N, parts, unique):
    cfg, db_np, bt, ts, batch = _run_step(dev, B, N, parts, unique)
    if unique:
        U = batch["src_unique"].U
        assert U < B * 16
    step_parity.record_pools(ts.models)
    loss, T = ts.forward(batch)
    got_terms = {k: float(T[k].detach()) for k in TERMS}
    out = T["_out"].detach()
    loss.backward()
    label = f"B={B} N={N} k={parts} unique={unique}"
    rgrads32 = _oracle_floor((B, N, parts), cfg, db_np, bt)
    choices = step_parity.gpu_pool_choices(ts.models, batch, unique)
    vals = step_parity.gpu_pool_values(ts.models, batch, unique)
    rterms, rout, rgrads, rpool = _oracle64(cfg, db_np, bt, choices, out.cpu(), vals)
    step_parity.tie_report(rpool, label)
    step_parity.check_loss_terms(got_terms, rterms, label)
    o = out.cpu()
    assert (o - rout).abs().max().item() <= 1e-4 * rout.abs().max().item()
    n, _ = step_parity.check_grads(ts.models, rgrads, label, ref32=rgrads32)
    assert n >= 145
    _check_step_nn(out, batch, cfg)
    return got_terms


def _check_step_nn(out, batch, cfg):
    """The chamfer full and part families of the step, re-run through the ragged NN kernel on the
    step's own deformed shape and segment tables, bit-exact vs the C oracle on the same inputs."""
    from loss.chamfer_loss import _full_segments
    from ured_hip.nn import nn_segments
    from ured_hip.ops import build_parts
    x = batch["x"]
    B, N, _ = x.shape
    S = out.shape[1]
    P = cfg["MAX_NUM_PARTS"]
    parts = build_parts(batch["labels"], x, P)
    k = parts.k
    segs = _full_segments(B, S, N, k, x.device, 1024)
    slot = torch.arange(P, device=x.device)
    valid = slot.unsqueeze(0) < k.unsqueeze(1)
    a_off = (torch.arange(B, device=x.device) * S).unsqueeze(1) + slot.unsqueeze(0) * 1024
    a_len = torch.where(valid, torch.full_like(a_off, 1024), torch.zeros_like(a_off))
    b_off = parts.off[:-1].view(B, P).long()
    b_len = torch.where(valid, parts.counts, torch.zeros_like(parts.counts))
    psegs = torch.stack([a_off, a_len, b_off, b_len], -1).view(B * P, 4).int()
    for a, b, sg, ma in ((out, x, segs, S), (out, parts.x_sorted, psegs, 1024)):
        a, b = a.contiguous(), b.contiguous()
        with torch.no_grad():
            da, ia, db, ib = nn_segments(a, b, sg, ma, N, 3)
        rda, ria, rdb, rib = nn_ref.nn_seg_fwd(a.cpu().numpy(), b.cpu().numpy(), sg.cpu().numpy())
        np.testing.assert_array_equal(ia.reshape(-1).cpu().numpy(), ria)
        np.testing.assert_array_equal(ib.reshape(-1).cpu().numpy(), rib)
        np.testing.assert_array_equal(da.reshape(-1).cpu().numpy(), rda)
        np.testing.assert_array_equal(db.reshape(-1).cpu().numpy(), rdb)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("unique", [True, False], ids=["unique_sources", "all_slots"])
@pytest.mark.parametrize("parts", [4, 16], ids=["k4", "k16"])
def test_config2_train_step_full_size(dev, parts, unique):
    terms = _check_step(dev, 16, 2048, parts, unique)
    print(f"\nconfig2 k={parts} unique={unique}: all_loss {terms['all_loss']:.6f}")


@pytest.mark.timeout(900)
def test_config5_train_step_4096_points(dev):
    terms = _check_step(dev, 8, 4096, 4, True)
    print(f"\nconfig5 bs=8 N=4096: all_loss {terms['all_loss']:.6f}")


@pytest.mark.timeout(900)
def test_config3_inference_full_size(dev):
    """engine/test.py inference at bs=16, 2048 points, C=512 over 512 sources vs ured_ref.infer
    (float64). Retrieval indices bit-exact outside top-2 gaps < 1e-6, and where a near-tie flipped
    a pick, the GPU's source is within 1e-6 of the float64 maximum similarity. Chamfer and
    DeformNet params of EVERY sample within 1e-4 / 1e-3: the oracle deforms the GPU's picks
    (ured_ref.infer(retrieved=...)), so a flipped near-tie is compared too, not skipped."""
    from dataset import synthetic
    from train_utils.load_sources import SourceDB
    from engine.train import get_models, batch_to_device
    from engine.test import infer
    _threads()
    cfg = _cfg(batch_size=16)
    dbn = synthetic.make_source_db(NS, seed=11)
    bt = synthetic.make_batch(16, 2048, NS, parts=[2, 3, 4, 5, 6, 7, 8, 16, 4, 4, 3, 9, 12, 1, 5, 4], seed=12)
    db = SourceDB(dbn["src_points"], dbn["src_mats"], dbn["src_default_param"], dbn["src_sem"], dev)
    models, _, _ = get_models(cfg, dev)
    P, _ = _params64(cfg, seed=5)
    P64 = {}
    for name, sd in P.items():
        sd = {k: (v + 0.05 if "running_var" in k else v) for k, v in sd.items()}   # non-trivial eval stats
        models[name].load_state_dict(sd, strict=True)
        P64[name] = {k: (v.double() if v.dtype.is_floating_point else v) for k, v in sd.items()}
    r = infer(models, db, batch_to_device(bt, dev), cfg)
    ob = {"src_points": torch.from_numpy(dbn["src_points"]).double(),
          "src_mats": torch.from_numpy(dbn["src_mats"]).double(),
          "src_sem": torch.from_numpy(dbn["src_sem"]), "x": torch.from_numpy(bt["x"]).double(),
          "labels": torch.from_numpy(bt["labels"]).double(), "tgt_sem": torch.from_numpy(bt["tgt_sem"])}
    R = ured_ref.infer(P64, ob, cfg)
    got, ref = r["retrieved"].cpu(), R["retrieved"]
    valid = ref >= 0
    near = (R["sim_top2_gap"] < 1e-6) & valid
    mism = (got != ref) & ~near
    flips = int(((got != ref) & near).sum())
    step_parity.report(f"\nconfig3: {int(valid.sum())} retrievals, {int(near.sum())} near-ties (gap < 1e-6), {flips} flipped")
    assert int(mism.sum()) == 0, f"{int(mism.sum())} retrieval mismatches outside near-ties"
    # a flipped pick is a near-optimal source in float64 terms
    sim = R["sim"]
    pick = sim.gather(-1, got.clamp(min=0).long().unsqueeze(-1)).squeeze(-1)
    loss_of_pick = (sim.max(-1).values - pick)[valid]
    assert float(loss_of_pick.max()) < 1e-6, f"a GPU pick is {float(loss_of_pick.max()):.3e} below the best similarity"
    # deformation of the GPU's picks, every sample
    R2 = R if flips == 0 else ured_ref.infer(P64, ob, cfg, retrieved=got)
    np.testing.assert_allclose(r["cd"].cpu().double().numpy(), R2["cd"].numpy(), rtol=1e-4)
    np.testing.assert_allclose(r["params"].cpu().double().numpy(), R2["params"].numpy(), rtol=1e-3, atol=1e-5)


@pytest.mark.timeout(600)
def test_nn_64x4096x4096(dev):
    """Config 5's NN shape through the dense drop-in: bit-exact vs the C oracle on 2 x 4096 sampled
    query rows (full candidate sets); on every row of both directions, the returned distance is
    the fp32 contract distance to the returned index and equals the float64 minimum within fp32
    rounding (no better candidate was missed)."""
    from ured_hip import nn as unn
    g = torch.Generator().manual_seed(5)
    B, n = 64, 4096
    p1 = torch.rand(B, n, 3, generator=g)
    p2 = torch.rand(B, n, 3, generator=g)
    a, b = p1.to(dev), p2.to(dev)
    d1, d2, i1, i2 = unn.nn_dense(a, b)
    assert ((i1 >= 0) & (i1 < n)).all() and ((i2 >= 0) & (i2 < n)).all()
    rng = np.random.Generator(np.random.PCG64(6))
    for q, r, d, i in ((p1, p2, d1, i1), (p2, p1, d2, i2)):
        bs = rng.integers(0, B, size=4096)
        rows = rng.integers(0, n, size=4096)
        for bb in np.unique(bs):
            sel = rows[bs == bb]
            rd, ri = nn_ref.nn_dir(q[bb, sel].numpy(), r[bb].numpy())
            np.testing.assert_array_equal(i[bb, sel].cpu().numpy(), ri)
            np.testing.assert_array_equal(d[bb, sel].cpu().numpy(), rd)
        qd, rd_ = q.to(dev).double(), r.to(dev).double()
        for bb in range(B):
            full = torch.cdist(qd[bb], rd_[bb]).square()
            mn = full.min(dim=1).values
            at = full.gather(1, i[bb].long().unsqueeze(1)).squeeze(1)
            tol = 2.4e-7 * mn + 1e-12
            assert ((at - mn).abs() <= 4 * tol + 1e-9).all(), f"batch {bb}: a closer candidate was missed"
            assert ((d[bb].double() - at).abs() <= 4 * tol + 1e-9).all(), f"batch {bb}: dist != |p - q[idx]|^2"
