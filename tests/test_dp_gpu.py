"""DataParallelStep end to end on the GPU box: 2 ranks (gloo — RCCL needs one GPU per rank
and the test box has one) each run the real HIP train step on its own shard; after
reduce_gradients every rank must hold the average of the ranks' local gradients, the
ranks' parameters stay identical after the Adam step. Then four full DataParallelSteps
(epochs 0, 0, 1, 1 with init_p_m_loss = 0: re_residual_net_full joins at epoch 1) with the
all-reduce buckets issued from backward's gradient hooks must leave exactly (bitwise) the
parameters of the same steps with the reduction done after backward."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG_DIR, ROOT

pytestmark = pytest.mark.gpu

CFG = {"source_latent_dim": 64, "target_latent_dim": 64, "sem_latent_dim": 16, "MAX_NUM_PARTS": 16,
       "alpha": 0.1, "use_chamfer_loss": 30.0, "use_chamfer_part_loss": 1.0, "use_symmetry_loss": 30.0,
       "use_contrast_loss": 0.5, "use_param_loss": 0.0, "init_p_m_loss": -1, "use_residuals_reg": 3.0,
       "use_recon": 30.0, "batch_size": 2, "device": "cuda", "optimizer": "adam", "learning_rate": 1e-3,
       "weight_decay": 5e-4, "lr_stepsize": 3, "lr_decay": 0.5, "momentum": 0.9}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    for p in (ROOT, PKG_DIR):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {"rank": rank, "avg": False, "same_params": False}
    try:
        from dataset import synthetic
        from engine.dp import DataParallelStep
        from engine.train import batch_to_device
        from oracle import ured_ref
        from train_utils.load_sources import SourceDB
        dev = torch.device("cuda", 0)
        dbn = synthetic.make_source_db(24, seed=3)
        db = SourceDB(dbn["src_points"], dbn["src_mats"], dbn["src_default_param"], dbn["src_sem"], dev)
        step = DataParallelStep(CFG, db, dev)
        for name, sd in ured_ref.make_params(CFG, seed=7).items():
            step.models[name].load_state_dict(sd, strict=True)
        batch = batch_to_device(synthetic.make_batch(2, 128, 24, parts=[3, 2], seed=40 + rank), dev)
        step.optimizer.zero_grad(set_to_none=True)
        loss, _ = step.forward(batch)
        loss.backward()
        local = {id(p): p.grad.detach().clone() for p in step.params if p.grad is not None}
        step.reduce_gradients()
        ok = True
        for p in step.params:
            if p.grad is None:
                continue
            allg = [torch.empty_like(local[id(p)]) for _ in range(world)]
            dist.all_gather(allg, local[id(p)])
            ok &= torch.allclose(p.grad, torch.stack(allg).mean(0), rtol=1e-5, atol=1e-7)
        res["avg"] = bool(ok)
        step.clip_and_step()
        w = step.models["src_encoder_all"].fuse_sem[0].weight.detach().clone()
        allw = [torch.empty_like(w) for _ in range(world)]
        dist.all_gather(allw, w)
        res["same_params"] = bool(torch.equal(allw[0], allw[1]))
        cfg = dict(CFG, init_p_m_loss=0)
        sa = DataParallelStep(cfg, db, dev, bucket_mb=0.2)   # overlapped (default for world > 1)
        sb = DataParallelStep(cfg, db, dev, overlap=False)
        for s_ in (sa, sb):
            for name, sd in ured_ref.make_params(CFG, seed=7).items():
                s_.models[name].load_state_dict(sd, strict=True)
        launched = []
        for ep in (0, 0, 1, 1):
            sa.step(batch, ep)
            sb.step(batch, ep)
            launched.append(sa.reducer.num_buckets)
        same = True
        for name in sa.models:
            pb = dict(sb.models[name].named_parameters())
            for k, p in sa.models[name].named_parameters():
                same &= bool(torch.equal(p.detach(), pb[k].detach()))
        res["overlap_equal"] = same
        res["buckets"] = launched
        torch.cuda.synchronize()
    finally:
        q.put(res)
        dist.destroy_process_group()


def test_dp_two_ranks_one_gpu(dev):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r["avg"], r
        assert r["same_params"], r
        assert r["overlap_equal"], r
        assert all(n > 1 for n in r["buckets"]), r
