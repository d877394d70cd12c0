"""Data-parallel plumbing on CPU with gloo, world_size 2 (127.0.0.1 rendezvous):
bucketed gradient averaging and the contrastive loss's cross-rank all_gather semantics
(loss/contrast_loss.py:35-102: labels offset by rank, gathered copies carry no gradient)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG_DIR, ROOT


def _free_port():
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
    ok_avg = ok_con = False
    try:
        from engine.dp import allreduce_gradients, make_buckets
        from loss.contrast_loss import compute_contrast_loss_loss
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.ReLU(), torch.nn.Linear(5, 3),
                                    torch.nn.Linear(4, 4))          # last layer unused: grad None
        x = torch.randn(6, 7, generator=torch.Generator().manual_seed(rank + 1))
        model[2](model[1](model[0](x))).pow(2).sum().backward()
        local = [p.grad.clone() if p.grad is not None else None for p in model.parameters()]
        buckets = make_buckets(list(model.parameters()), bucket_elems=20)
        allreduce_gradients(buckets, world)
        gathered = []
        for g in local:
            if g is None:
                gathered.append(None)
                continue
            allg = [torch.empty_like(g) for _ in range(world)]
            dist.all_gather(allg, g)
            gathered.append(torch.stack(allg).mean(0))
        ok_avg = all((p.grad is None and g is None) or torch.allclose(p.grad, g, atol=1e-6)
                     for p, g in zip(model.parameters(), gathered))
        # contrast loss: 2 samples x 3 part slots per rank
        gen = torch.Generator().manual_seed(10 + rank)
        t = torch.randn(2, 3, 8, generator=gen, requires_grad=True)
        s = torch.randn(2, 3, 8, generator=gen, requires_grad=True)
        lab = torch.tensor([[1, 1, -1], [1, -1, -1]])
        loss = compute_contrast_loss_loss(t, s, lab)
        loss.backward()
        # restated: logits vs all ranks' sources, labels offset by rank, no grad to other ranks
        te = torch.nn.functional.normalize(t.detach().reshape(6, 8), dim=-1)
        se = torch.nn.functional.normalize(s.detach().reshape(6, 8), dim=-1)
        alls = [torch.empty_like(se) for _ in range(world)]
        dist.all_gather(alls, se)
        labels = 6 * rank + torch.arange(6)
        labels[lab.reshape(-1) == -1] = -1
        ref = torch.nn.functional.cross_entropy((1 / 0.07) * te @ torch.cat(alls).t(), labels, ignore_index=-1)
        ok_con = abs(loss.item() - ref.item()) < 1e-4 and (s.grad is None or s.grad.abs().sum().item() == 0.0)
    finally:
        q.put((rank, ok_avg, ok_con))
        dist.destroy_process_group()


def test_dp_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for rank, ok_avg, ok_con in res:
        assert ok_avg, f"rank {rank}: gradient average mismatch"
        assert ok_con, f"rank {rank}: contrastive all_gather semantics mismatch"


def _reducer_worker(rank, world, port, q):
    """FlatGradReducer (engine/dp.py) over a FlatAdam layout on CPU tensors (the layout,
    bucketing, hooks and collectives are host logic; only FlatAdam.step needs the GPU)."""
    import sys
    for p in (ROOT, PKG_DIR):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {"rank": rank, "ok": [], "overlapped": [], "buckets": []}
    try:
        from engine.dp import FlatGradReducer
        from ured_hip.optim import FlatAdam
        torch.manual_seed(0)
        mods = [torch.nn.Linear(6, 9), torch.nn.Linear(9, 9), torch.nn.Linear(9, 4), torch.nn.Linear(4, 4),
                torch.nn.Linear(3, 3)]                    # mods[3]: joins at step 2; mods[4]: never used
        ref = [torch.nn.Linear(1, 1) for _ in mods]
        for r, m in zip(ref, mods):                       # an identical copy for the local gradients
            r.weight = torch.nn.Parameter(m.weight.detach().clone())
            r.bias = torch.nn.Parameter(m.bias.detach().clone())
        params = [p for m in mods for p in m.parameters()]
        opt = FlatAdam(params, [list(mods[0].parameters()) + list(mods[1].parameters()),
                                list(mods[2].parameters()) + list(mods[3].parameters()) + list(mods[4].parameters())])
        red = FlatGradReducer(opt, params, world, bucket_elems=40, overlap=True, last_elems=12)

        def fwd(ms, x, use3):
            h = ms[2](torch.relu(ms[1](torch.relu(ms[0](x)))))
            if use3:
                h = ms[3](h)
            return h.pow(2).sum()

        for it in range(4):
            use3 = it >= 2
            x = torch.randn(5, 6, generator=torch.Generator().manual_seed(100 * it + rank))
            for p in [p for r in ref for p in r.parameters()]:
                p.grad = None
            fwd(ref, x, use3).backward()
            local = [p.grad.clone() if p.grad is not None else None for r in ref for p in r.parameters()]
            opt.zero_grad(set_to_none=True)
            nb_before = red.num_buckets
            red.issued.clear()
            red.begin()
            fwd(mods, x, use3).backward()
            res["overlapped"].append(red._fb is not None and any(b.launched for b in red._fb))
            red.finish()
            ok = True
            for p, g in zip(params, local):
                if g is None:
                    ok &= p.grad is None
                    continue
                allg = [torch.empty_like(g) for _ in range(world)]
                dist.all_gather(allg, g)
                ok &= bool(torch.allclose(p.grad, torch.stack(allg).mean(0), atol=1e-6))
                ok &= p.grad.data_ptr() >= opt.flat_grad.data_ptr()      # a view of the flat buffer
            res["ok"].append(ok)
            res["buckets"].append(sum(len(b.params) for b in red._fb))
            # buckets are all-reduced strictly in index order, every one of them once
            res["order_ok"] = res.get("order_ok", True) and red.issued == list(range(nb_before))
            res.setdefault("nbuckets", []).append(red.num_buckets)
            # the last bucket (the one left after backward) is cut at ~last_elems
            fb = red._fb
            res["last_small"] = res.get("last_small", True) and (
                len(fb) < 2 or sum(p.numel() for p in fb[-1].params[1:]) < red.last_elems)
            with torch.no_grad():                          # the same update on both copies
                for p, r in zip(params, [p for r in ref for p in r.parameters()]):
                    if p.grad is not None:
                        p.sub_(0.01 * p.grad)
                        r.copy_(p)
    finally:
        q.put(res)
        dist.destroy_process_group()


def test_flat_grad_reducer_gloo_world2():
    """Bucketed all-reduce issued from backward's gradient hooks: every step leaves the rank
    average in the flat gradient; from the second step on buckets are issued during backward;
    a parameter that starts getting a gradient later (step 3) is reduced and then bucketed."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_reducer_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for r in res:
        assert r["ok"] == [True] * 4, r
        assert r["overlapped"] == [False, True, True, True], r
        # bucketed parameters: the one joining at step 3 is bucketed from then on
        assert r["nbuckets"][0] > 1 and r["buckets"][3] > r["buckets"][1], r
        assert r["order_ok"] and r["last_small"], r
