"""Data-parallel training at the multi-GPU BASELINE configurations' per-rank shapes, on the one
GPU of the test box (gloo carries the collectives: RCCL needs one GPU per rank).

config 4  storagefurniture, global bs 32 over 4 ranks: 4 ranks x bs 8, 2048 points, C=512
config 5  chair, global bs 64 over 8 ranks, 4096-point clouds: 8 ranks x bs 8, 4096 points

Each rank runs the real HIP train step (engine/dp.py DataParallelStep, the configuration of
config/config_train_test.json) on its own shard for two steps; the second step's gradient
all-reduce buckets are issued from backward's hooks (the first builds the bucket layout).
Checked on every rank (DDP semantics):
  * after reduce_gradients, every gradient equals the mean of the ranks' local gradients
    within 1e-5 of the mean magnitude sum(|g_r|)/world element by element (the collective sums
    in its own order; a fp32 sum of `world` terms errs relative to the sum of magnitudes);
  * after the Adam step the parameters are bitwise identical across ranks;
  * the losses are finite and differ across ranks (each rank saw its own shard).
The single-rank numerics of the same step are covered by tests/test_fullsize_gpu.py.
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


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, bs, npts, q):
    import sys
    for p in (ROOT, PKG_DIR):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {"rank": rank}
    try:
        from dataset import synthetic
        from engine.dp import DataParallelStep
        from engine.train import batch_to_device
        from train_utils.load_sources import SourceDB
        with open(os.path.join(PKG_DIR, "config", "config_train_test.json")) as f:
            cfg = json.load(f)
        cfg.update(device="cuda", log_every=0, batch_size=bs)
        dev = torch.device("cuda", 0)
        dbn = synthetic.make_source_db(512, seed=3)
        db = SourceDB(dbn["src_points"], dbn["src_mats"], dbn["src_default_param"], dbn["src_sem"], dev)
        torch.manual_seed(11)                      # identical initial weights on every rank
        step = DataParallelStep(cfg, db, dev)
        ok_avg, losses, worst = True, [], 0.0
        for it in range(2):
            batch = batch_to_device(synthetic.make_batch(bs, npts, 512, parts=4, seed=100 * it + rank), dev)
            # the rank's local gradient first (hooks not armed: nothing is reduced), then the same
            # step again with the reduction (gradients land in the flat buffer that the hooks
            # all-reduce in place during backward, as DDP does; training-mode BN makes the second
            # forward's values identical)
            step.optimizer.zero_grad(set_to_none=True)
            loss, _ = step.forward(batch, 1)
            loss.backward()
            local = {id(p): p.grad.detach().clone() for p in step.params if p.grad is not None}
            step.optimizer.zero_grad(set_to_none=True)
            loss, _ = step.forward(batch, 1)
            if step.reducer is not None:
                step.reducer.begin()               # step 2: buckets all-reduced from backward's hooks
            loss.backward()
            step.reduce_gradients()
            for p in step.params:
                if id(p) not in local:
                    continue
                allg = [torch.empty_like(local[id(p)]) for _ in range(world)]
                dist.all_gather(allg, local[id(p)])
                mean = sum(allg[1:], allg[0].clone()) / world
                # the collective's summation order is its own (ring / halving-doubling): the error
                # bound of a fp32 sum of `world` terms is relative to the sum of magnitudes
                mag = sum(a.abs() for a in allg) / world
                err = float(((p.grad - mean).abs() / (mag + 1e-30)).max())
                if err > worst:
                    name = next(f"{m}.{k}" for m in step.models for k, q in step.models[m].named_parameters() if q is p)
                    i = int(((p.grad - mean).abs() / (mag + 1e-30)).argmax())
                    res["worst_at"] = (it, name, i, float(p.grad.reshape(-1)[i]), float(mean.reshape(-1)[i]),
                                       float(mag.reshape(-1)[i]), [float(a_.reshape(-1)[i]) for a_ in allg])
                worst = max(worst, err)
                ok_avg &= err <= 1e-5
            step.clip_and_step()
            losses.append(float(loss))
        res["avg"], res["worst_rel_err"] = ok_avg, worst
        same = True
        for name in sorted(step.models):
            for k, p in step.models[name].named_parameters():
                allp = [torch.empty_like(p.detach()) for _ in range(world)]
                dist.all_gather(allp, p.detach().contiguous())
                same &= all(torch.equal(allp[0], a) for a in allp[1:])
        res["same_params"] = same
        res["losses"] = losses
        torch.cuda.synchronize()
    except Exception as e:                          # reported to the parent, which fails the test
        import traceback
        res["error"] = repr(e) + "\n" + traceback.format_exc()[-3000:]
    finally:
        q.put(res)
        dist.destroy_process_group()


# Hardware queues per rank process. Each HIP process opens up to GPU_MAX_HW_QUEUES (4 on the box)
# queues; eight ranks plus the test process on ONE card then ask the scheduler for ~36 queues,
# beyond what it maps at once, so it time-slices them with mid-kernel context save/restore — a
# regime that exists only in this one-GPU rehearsal (production runs one rank per GPU). Two per
# rank keeps the 8-rank rehearsal at the 4-rank one's queue count ("The multi-process
# fault").
# What this cap means for the evidence: the HSA_STATUS_ERROR_ILLEGAL_INSTRUCTION aborts of rounds
# 3 and 4 happened in the UNCAPPED 8-rank run (nine processes x 4 queues). With the cap, the
# 8-rank test no longer runs in that regime, so its green runs do not show that the round-5
# change (the compiler's LDS-DMA builtin issued ahead of the MFMAs) removed the cause; they show
# that the data-parallel step is correct at eight ranks. The memory-safety side is checked
# separately: the single-process suite on the bounds-checked build (tools/debug_bounds_suite.sh).
# URED_TEST_RANK_HW_QUEUES overrides the cap ("default": no cap, the r3 / r4 regime) for a
# deliberate diagnostic run; the suite's default keeps it.
RANK_HW_QUEUES = os.environ.get("URED_TEST_RANK_HW_QUEUES", "2")


def _run(world, bs, npts):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, bs, npts, q)) for r in range(world)]
    old = os.environ.get("GPU_MAX_HW_QUEUES")
    if RANK_HW_QUEUES != "default":
        os.environ["GPU_MAX_HW_QUEUES"] = RANK_HW_QUEUES     # inherited by the spawned ranks only
    try:
        for p in procs:
            p.start()
    finally:
        if old is None:
            os.environ.pop("GPU_MAX_HW_QUEUES", None)
        else:
            os.environ["GPU_MAX_HW_QUEUES"] = old
    res = [q.get(timeout=360) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert "error" not in r, r
        assert r["avg"], (r["rank"], r["worst_rel_err"], r.get("worst_at"), r)
        assert r["same_params"], r
        assert all(math.isfinite(v) for v in r["losses"]), r
    first = sorted(r["losses"][0] for r in res)
    assert first[0] != first[-1], "every rank computed the same loss: the shards were not distinct"
    print(f"world {world}: step-1 losses per rank {[round(r['losses'][0], 4) for r in sorted(res, key=lambda r: r['rank'])]}, "
          f"worst gradient-average error {max(r['worst_rel_err'] for r in res):.2e}")


@pytest.mark.timeout(400)
def test_config4_four_ranks_bs8_2048pts(dev):
    _run(4, 8, 2048)


@pytest.mark.timeout(400)
def test_config5_eight_ranks_bs8_4096pts(dev):
    _run(8, 8, 4096)
