"""Optional SyncBN (cfg["sync_bn"], ured_hip/syncbn.py): two ranks on half batches equal one rank
on the full batch — gloo carries the collectives, both ranks share the one GPU of the test box.

Each rank first computes the reference: a TrainStep without SyncBN on the FULL batch (4
samples), with the process group hidden from the contrastive loss (world 1). Then the
DataParallelStep with sync_bn on its half (2 samples; unique-source encoding with row
multiplicities, the default GPU path) and the gradient all-reduce. Checked (equal part counts
and valid sources, so every loss term is a plain mean over the samples):
  * every BatchNorm's running mean / var after the step's forward — the per-point BNs of the
    encoders and residual / reconstruction nets (ured_bn_stats / ured_bn_finalize_stats) and
    DeformNet's node BNs (ured_node_bn_fwd SyncBN modes) — equal the full batch's within 1e-5
    of the buffer's largest entry, and are BITWISE equal across the ranks (one merge, in rank
    order, on every rank); a control step without SyncBN on the same half batch deviates by
    > 1e-2 (its shard's statistics);
  * the forward outputs (deformed shapes, DeformNet parameters) of each rank's samples equal the
    full batch's rows within 1e-4 of the largest entry (measured: bitwise equal — the merged
    fp64 statistics round to the same fp32 values and the GEMM rows do not depend on the batch);
  * the mean over the ranks of every loss term equals the full batch's term within 2e-5;
  * after the gradient all-reduce every parameter gradient equals the full batch's within 1e-3
    in norm (the GEMMs reduce the halves in another fp32 order and the BN coefficients come
    from the merged fp64 sums); the conv biases that feed a training-mode BN have a true
    gradient of 0 and are checked to be rounding noise (step_parity.zero_true_grad).
The contrastive term is off here: under data parallelism its source codes are all-gathered
without the other ranks' gradient (the reference's all_gather, loss/contrast_loss.py), so its
gradient is not the full batch's whether or not BN is synchronised.
"""
import json
import math
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG_DIR, ROOT

pytestmark = pytest.mark.gpu

BS, NPTS = 4, 1024
TERMS = ("cd_loss_full", "cd_loss_part", "ref_cd_loss_full", "ref_cd_loss_part", "re_reg_loss_full", "reg_loss_full",
         "recon_loss_full", "recon_loss_src")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bn_buffers(models):
    out = {}
    for name in sorted(models):
        for k, b in models[name].named_buffers():
            if k.endswith(("running_mean", "running_var", "num_batches_tracked")):
                out[(name, k)] = b.detach().clone()
    return out


def _worker(rank, world, port, q):
    import sys
    for p in (ROOT, PKG_DIR):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {"rank": rank}
    try:
        import loss.contrast_loss as cl
        from dataset import synthetic
        from engine.dp import DataParallelStep
        from engine.train import TrainStep, batch_to_device
        from train_utils.load_sources import SourceDB
        from ured_hip import syncbn
        with open(os.path.join(PKG_DIR, "config", "config_train_test.json")) as f:
            cfg = json.load(f)
        cfg.update(device="cuda", log_every=0, use_contrast_loss=0.0)
        dev = torch.device("cuda", 0)
        dbn = synthetic.make_source_db(512, seed=3)
        db = SourceDB(dbn["src_points"], dbn["src_mats"], dbn["src_default_param"], dbn["src_sem"], dev)
        full = synthetic.make_batch(BS, NPTS, 512, parts=4, seed=21)
        half = {k: v[rank * BS // world:(rank + 1) * BS // world] for k, v in full.items()}

        # the reference: one rank, the full batch, no SyncBN (the contrastive loss sees world 1)
        hidden = cl.is_dist_avail_and_initialized
        cl.is_dist_avail_and_initialized = lambda: False
        try:
            torch.manual_seed(11)
            ref = TrainStep(dict(cfg, batch_size=BS, sync_bn=False), db, dev)
            assert not ref.sync_bn and not syncbn.active()
            ref.optimizer.zero_grad(set_to_none=True)
            lr_, Tr = ref.forward(batch_to_device(full, dev, num_sources=db.num_sources), 1)
            lr_.backward()
        finally:
            cl.is_dist_avail_and_initialized = hidden
        ref_bn = _bn_buffers(ref.models)
        ref_T = {k: float(Tr[k]) for k in TERMS if k in Tr}
        sl = slice(rank * BS // world, (rank + 1) * BS // world)
        ref_out, ref_par = Tr["_out"][sl].detach().clone(), Tr["_params"].view(BS, -1)[sl].detach().clone()
        ref_g = {(m, k): p.grad.detach().clone() for m in sorted(ref.models)
                 for k, p in ref.models[m].named_parameters() if p.grad is not None}

        # SyncBN over the two ranks, half a batch each
        torch.manual_seed(11)
        step = DataParallelStep(dict(cfg, batch_size=BS // world, sync_bn=True), db, dev)
        assert step.sync_bn and syncbn.active()
        step.optimizer.zero_grad(set_to_none=True)
        loss, T = step.forward(batch_to_device(half, dev, num_sources=db.num_sources), 1)
        bn = _bn_buffers(step.models)
        loss.backward()
        step.reduce_gradients()

        worst_bn, same_bn = 0.0, True
        for key, r in ref_bn.items():
            b = bn[key]
            if key[1].endswith("num_batches_tracked"):
                same_bn &= bool(torch.equal(b, r))
                continue
            worst_bn = max(worst_bn, float((b - r).abs().max() / r.abs().max().clamp(min=1e-30)))
            allb = [torch.empty_like(b) for _ in range(world)]
            dist.all_gather(allb, b.contiguous())
            same_bn &= all(torch.equal(allb[0], a) for a in allb[1:])
        res["bn_worst"], res["bn_same_across_ranks"], res["n_bn"] = worst_bn, same_bn, len(ref_bn)
        res["out_err"] = float((T["_out"].detach() - ref_out).abs().max() / ref_out.abs().max())
        res["par_err"] = float((T["_params"].detach().view(BS // world, -1) - ref_par).abs().max()
                               / ref_par.abs().max())
        terms = torch.tensor([float(T[k]) for k in ref_T], dtype=torch.float64)
        dist.all_reduce(terms)
        res["terms"] = {k: (float(v) / world, ref_T[k]) for k, v in zip(ref_T, terms)}
        import step_parity
        worst_g, missing, errs, zero_worst = 0.0, [], [], 0.0
        gmax = {m: max([float(g.abs().max()) for (mm, _), g in ref_g.items() if mm == m] + [1e-30])
                for m in step.models}
        for m in sorted(step.models):
            for k, p in step.models[m].named_parameters():
                r = ref_g.get((m, k))
                if r is None:
                    if p.grad is not None and float(p.grad.abs().max()) > 0:
                        missing.append((m, k, "extra"))
                    continue
                if p.grad is None:
                    missing.append((m, k, "none"))
                    continue
                if step_parity.zero_true_grad(m, k):
                    # a conv bias feeding a training-mode BN: its true gradient is 0, both are
                    # rounding noise (checked tiny against the module's largest gradient instead)
                    zero_worst = max(zero_worst, float(p.grad.abs().max()) / gmax[m], float(r.abs().max()) / gmax[m])
                    continue
                e = float((p.grad - r).norm() / r.norm().clamp(min=1e-30))
                errs.append((e, m, k, float(p.grad.norm()), float(r.norm())))
                worst_g = max(worst_g, e)
        res["grad_worst"], res["grad_missing"], res["n_grads"] = worst_g, missing, len(ref_g)
        res["grad_top"], res["zero_grad_worst"] = sorted(errs, reverse=True)[:6], zero_worst
        # control: the same half batch without SyncBN normalises with the shard's statistics
        del loss, T
        torch.manual_seed(11)
        local = DataParallelStep(dict(cfg, batch_size=BS // world, sync_bn=False), db, dev)
        assert not syncbn.active()
        with torch.no_grad():
            local.forward(batch_to_device(half, dev, num_sources=db.num_sources), 1)
        lbn = _bn_buffers(local.models)
        res["local_bn_dev"] = max(float((lbn[k] - r).abs().max() / r.abs().max().clamp(min=1e-30))
                                  for k, r in ref_bn.items() if not k[1].endswith("num_batches_tracked"))
        torch.cuda.synchronize()
    except Exception as e:                          # reported to the parent, which fails the test
        import traceback
        res["error"] = traceback.format_exc()
    finally:
        q.put(res)
        dist.destroy_process_group()


@pytest.mark.timeout(400)
def test_syncbn_two_half_batches_equal_full_batch(dev):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=360) for _ in procs], key=lambda r: r["rank"])
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert "error" not in r, r.get("error")
    for r in res:
        print(f"rank {r['rank']}: {r['n_bn']} BN buffers, worst {r['bn_worst']:.2e}; out {r['out_err']:.2e} "
              f"params {r['par_err']:.2e}; {r['n_grads']} grads, worst norm err {r['grad_worst']:.2e}; "
              f"without SyncBN the BN buffers deviate {r['local_bn_dev']:.2e}")
        for t in r["grad_top"]:
            print("   grad err %.2e %s %s |g| %.4g |ref| %.4g" % t)
        assert r["bn_same_across_ranks"], "BN statistics differ across ranks"
        assert r["bn_worst"] <= 1e-5, r["bn_worst"]
        assert r["local_bn_dev"] > 1e-2, r["local_bn_dev"]       # the control: shard statistics differ
        assert r["out_err"] <= 1e-4 and r["par_err"] <= 1e-4, (r["out_err"], r["par_err"])
        assert not r["grad_missing"], r["grad_missing"]
        assert r["grad_worst"] <= 1e-3, r["grad_worst"]
        assert r["zero_grad_worst"] <= 1e-3, r["zero_grad_worst"]
    for k, (got, exp) in res[0]["terms"].items():
        print(f"  {k}: ranks' mean {got:.7g} full batch {exp:.7g}")
        assert math.isfinite(got) and abs(got - exp) <= 2e-5 * abs(exp), (k, got, exp)
