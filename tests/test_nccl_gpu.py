"""The RCCL ("nccl") code paths of the data-parallel step on the one GPU of the test box: a
world-size-1 nccl process group with cfg["dp_force_collectives"], so every collective really goes
through RCCL (the bucketed gradient all-reduce issued from backward's hooks, the contrastive
all_gather), eagerly and captured INSIDE the replayed HIP graph (engine/graph.py: one graph, no
split at the collectives). A one-rank all-reduce / all-gather is the identity, so:
  * without the contrastive term (no gather) DataParallelStep eager and graph-replayed equal a
    plain TrainStep bitwise, losses and parameters;
  * with it (the gathered-codes contrast path instead of the loss head's own; differentiable
    gather, so that the source codes keep their contrastive gradient as in the single-process
    step — the reference's plain all_gather would drop it) eager == replay bitwise, and the
    losses match TrainStep to 1e-5 relative over the first three steps (a different fp32
    arithmetic path: Adam then amplifies the rounding differences of near-zero gradients, and
    the trajectories drift apart, ~1e-2 by the sixth step).
The same two steps with cfg["graph_inline_collectives"] = False take the path world > 1 uses by
default: segmented capture, the collectives run eagerly between graph segments on RCCL, the
gradient all-reduce after the replay; they must equal the plain / eager steps bitwise too.
Runs in a spawned process (its process group must not leak into the other tests)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from conftest import PKG_DIR, ROOT
from test_dp_gpu import CFG

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(port, q):
    import sys
    for p in (ROOT, PKG_DIR):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    res = {}
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        res["backend"] = dist.get_backend()
        from dataset import synthetic
        from engine.dp import DataParallelStep
        from engine.graph import GraphedStep
        from engine.train import TrainStep, batch_to_device
        from oracle import ured_ref
        from train_utils.load_sources import SourceDB
        dbn = synthetic.make_source_db(24, seed=3)
        db = SourceDB(dbn["src_points"], dbn["src_mats"], dbn["src_default_param"], dbn["src_sem"], dev)
        batches = [batch_to_device(synthetic.make_batch(2, 128, 24, parts=[3, 2], seed=60 + i), dev) for i in range(3)]

        def make(cls, cfg):
            s = cls(cfg, db, dev)
            for name, sd in ured_ref.make_params(cfg, seed=7).items():
                s.models[name].load_state_dict(sd, strict=True)
            return s

        def run(step, n=6):
            return [float(step.step(batches[i % 3])["all_loss"]) for i in range(n)]

        def params(step):
            return {(m, k): p.detach().clone() for m in step.models for k, p in step.models[m].named_parameters()}

        cfg1 = dict(CFG, use_contrast_loss=0.0, cuda_graph=True)
        cfg2 = dict(CFG, cuda_graph=True, differentiable_gather=True)
        ref1 = make(TrainStep, cfg1)
        l_ref1, p_ref1 = run(ref1), params(ref1)
        ref2 = make(TrainStep, cfg2)
        l_ref2 = run(ref2)
        force = {"dp_force_collectives": True}
        e1 = make(DataParallelStep, dict(cfg1, **force))
        assert e1.collect and e1.reducer is not None
        l_e1, p_e1 = run(e1), params(e1)
        g1 = GraphedStep(make(DataParallelStep, dict(cfg1, **force)))
        l_g1, p_g1 = run(g1), params(g1)
        ent = next(iter(g1.graphs.values()))
        res["inline"] = ent[1].inline and bool(ent[3]) and len(ent[1].graphs) == 1 and not ent[1].collectives
        res["buckets"] = g1.inner.reducer.num_buckets
        res["eager1_eq_train"] = l_e1 == l_ref1 and all(torch.equal(p_e1[k], p_ref1[k]) for k in p_ref1)
        res["graph1_eq_train"] = l_g1 == l_ref1 and all(torch.equal(p_g1[k], p_ref1[k]) for k in p_ref1)
        e2 = make(DataParallelStep, dict(cfg2, **force))
        l_e2, p_e2 = run(e2), params(e2)
        g2 = GraphedStep(make(DataParallelStep, dict(cfg2, **force)))
        l_g2, p_g2 = run(g2), params(g2)
        res["graph2_eq_eager2"] = l_g2 == l_e2 and all(torch.equal(p_g2[k], p_e2[k]) for k in p_e2)
        res["contrast_rel"] = [abs(a - b) / abs(b) for a, b in zip(l_e2, l_ref2)]
        # the world > 1 default: segmented capture, RCCL collectives eagerly between the graph
        # segments — the all_gather and each gradient bucket's all-reduce, issued from the
        # replayed backward between its segments (forced here at world size 1)
        seg = {"graph_inline_collectives": False}
        g3 = GraphedStep(make(DataParallelStep, dict(cfg1, **force, **seg)))
        l_g3, p_g3 = run(g3), params(g3)
        g4 = GraphedStep(make(DataParallelStep, dict(cfg2, **force, **seg)))
        l_g4, p_g4 = run(g4), params(g4)
        ent4 = next(iter(g4.graphs.values()))
        res["segmented"] = (not ent4[1].inline and bool(ent4[3])
                            and len(ent4[1].graphs) == len(ent4[1].collectives) + 1 >= 3)
        res["seg1_eq_train"] = l_g3 == l_ref1 and all(torch.equal(p_g3[k], p_ref1[k]) for k in p_ref1)
        res["seg2_eq_eager2"] = l_g4 == l_e2 and all(torch.equal(p_g4[k], p_e2[k]) for k in p_e2)
        res["losses"] = (l_ref1[:2], l_e1[:2], l_g1[:2])
        torch.cuda.synchronize()
    except Exception as e:
        import traceback
        res["error"] = repr(e) + "\n" + traceback.format_exc()[-3000:]
    finally:
        q.put(res)
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_nccl_world1_eager_and_captured(dev):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_port(), q))
    p.start()
    r = q.get(timeout=280)
    p.join(timeout=60)
    assert "error" not in r, r["error"]
    assert r["backend"] == "nccl"
    assert r["inline"], r                      # one graph, the collectives captured in it
    assert r["buckets"] >= 1, r
    assert r["eager1_eq_train"], r
    assert r["graph1_eq_train"], r
    assert r["graph2_eq_eager2"], r
    assert max(r["contrast_rel"][:3]) <= 1e-5, r
    assert r["segmented"], r                   # split at the all_gather: 2+ graphs, eager collectives
    assert r["seg1_eq_train"], r
    assert r["seg2_eq_eager2"], r
    print(f"\nnccl world 1: {r['buckets']} gradient buckets captured; contrast path rel dev per step "
          f"{['%.1e' % v for v in r['contrast_rel']]}")
