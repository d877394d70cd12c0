"""Graph replay of the DATA-PARALLEL step (engine/graph.py with world > 1): the captured step is a
chain of graphs split at its collectives (the contrastive loss's all_gather; with SyncBN every
BN statistics exchange) and at the gradient buckets the backward's hooks all-reduce, replayed
with the collectives issued eagerly between the segments (ured_hip/collective.py: each bucket's
all-reduce right after the segment that wrote it, overlapping the rest of the backward; the
waits and the 1/world scaling at the end of the captured region), then the update graph.

gloo world 2, both ranks on the one GPU of the test box, each rank its own batches. Per rank, an
eager DataParallelStep and a GraphedStep over another DataParallelStep (same initial weights)
take the same 4 steps (one capture, three replays): the losses of every step and all parameters
and BN buffers after them are BITWISE equal between the two modes — the replay runs the eager
step's kernels, and the reductions sum the same two addends — and the parameters are bitwise
equal across the ranks. Also: every active gradient is its flat-gradient view after capture
(the torch-produced gradients are gathered inside the captured region, so the all-reduce after
a replay reads this step's gradients)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
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


def _worker(rank, world, port, sync_bn, q):
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
        from engine.graph import GraphedStep
        from engine.train import batch_to_device
        from train_utils.load_sources import SourceDB
        from ured_hip import collective
        dev = torch.device("cuda", 0)
        cfg = dict(CFG, cuda_graph=True, sync_bn=sync_bn)
        dbn = synthetic.make_source_db(24, seed=3)
        db = SourceDB(dbn["src_points"], dbn["src_mats"], dbn["src_default_param"], dbn["src_sem"], dev)
        # one padded distinct-part count for all batches: one graph, three replays
        batches = [batch_to_device(synthetic.make_batch(2, 128, 24, parts=[3, 2], seed=100 * rank + i), dev, 24,
                                   bucket=16) for i in range(4)]
        # small buckets, so that the captured backward is split at several bucket all-reduces
        torch.manual_seed(5)
        a = DataParallelStep(cfg, db, dev, bucket_mb=0.5, last_bucket_mb=0.1)
        torch.manual_seed(5)
        b = DataParallelStep(cfg, db, dev, bucket_mb=0.5, last_bucket_mb=0.1)
        g = GraphedStep(a)
        same_loss = True
        orders, eager_orders = [], []
        for i, bt in enumerate(batches):
            a.reducer.issued.clear()
            b.reducer.issued.clear()
            la = g.step(bt)["all_loss"].clone()
            lb = b.step(bt)["all_loss"]
            orders.append(list(a.reducer.issued))
            eager_orders.append(list(b.reducer.issued))
            same_loss &= bool(torch.equal(la, lb))
        res["orders"], res["eager_orders"], res["nbuckets"] = orders, eager_orders, a.reducer.num_buckets
        res["deferred"] = list(a.reducer.deferred)
        ent = next(iter(g.graphs.values()))
        res["segments"], res["collectives"] = len(ent[1].graphs), len(ent[1].collectives)
        res["ngraphs"] = len(g.graphs)
        assert collective._split is None
        opt = a.optimizer
        res["grads_are_views"] = all(p.grad.data_ptr() == v.data_ptr()
                                     for p, v, act in zip(opt.params_all, opt._gviews, opt._active) if act)
        same_mode, n = True, 0
        for name in sorted(a.models):
            for (k, pa), (_, pb) in zip(a.models[name].state_dict().items(), b.models[name].state_dict().items()):
                if not torch.equal(pa, pb):
                    same_mode = False
                    res.setdefault("differ", []).append((name, k, float((pa.double() - pb.double()).abs().max())))
                n += 1
        res["same_loss"], res["same_mode"], res["n_tensors"] = same_loss, same_mode, n
        same_rank = True
        for name in sorted(a.models):
            for k, p in a.models[name].named_parameters():
                allp = [torch.empty_like(p.detach()) for _ in range(world)]
                dist.all_gather(allp, p.detach().contiguous())
                same_rank &= all(torch.equal(allp[0], x) for x in allp[1:])
        res["same_rank"] = same_rank
        torch.cuda.synchronize()
    except Exception:
        import traceback
        res["error"] = traceback.format_exc()
    finally:
        q.put(res)
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("sync_bn", [False, True], ids=["local_bn", "sync_bn"])
def test_graph_dp_replay_equals_eager(dev, sync_bn):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, sync_bn, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in procs], key=lambda r: r["rank"])
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert "error" not in r, r.get("error")
    for r in res:
        print(f"rank {r['rank']}: {r['ngraphs']} graph(s), {r['segments']} segments / {r['collectives']} "
              f"collectives, {r['nbuckets']} buckets, {len(r['deferred'])} bucket hooks off the capture stream, "
              f"{r['n_tensors']} tensors compared")
        assert r["ngraphs"] == 1
        assert r["collectives"] >= 1 and r["segments"] == r["collectives"] + 1
        # the gradient buckets are all-reduced from the replayed step, between its backward
        # segments, strictly in bucket order (step 0 runs eagerly before any bucket exists, then
        # is captured: its collectives are recorded, not issued); the eager steps issue the same
        nb = r["nbuckets"]
        assert nb >= 3, r
        assert r["orders"][0] == [] and all(o == list(range(nb)) for o in r["orders"][1:]), r["orders"]
        assert r["eager_orders"][0] == [] and all(o == list(range(nb)) for o in r["eager_orders"][1:])
        # at least one split per bucket hook beyond the forward's all_gather (several buckets can
        # fill at one hook and share a split)
        assert r["collectives"] >= 3, r
        if sync_bn:
            assert r["collectives"] > 20           # every BN layer's exchange, forward and backward
        assert r["grads_are_views"]
        assert r["same_loss"], r
        assert r["same_mode"], r.get("differ", [])[:8]
        assert r["same_rank"]
