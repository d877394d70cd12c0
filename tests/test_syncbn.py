"""SyncBN host logic (ured_hip/syncbn.py) on CPU over gloo, world 2: the rank-order Chan merge of
per-rank fp64 (count, mean, M2) equals the statistics of the concatenated rows, identically on
every rank, and the backward sums add up. The GPU kernels around it (ured_bn_stats,
ured_bn_finalize_stats, ured_bn_bwd_sums, the node BN SyncBN modes) are covered by
tests/test_syncbn_gpu.py."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG_DIR, ROOT


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rows(rank):
    g = np.random.default_rng(7 + rank)
    n = (37, 101)[rank]                           # unequal shards
    return g.standard_normal((n, 2, 5)) * (1 + 3 * rank) + rank


def _worker(rank, world, port, q):
    import sys
    for p in (ROOT, PKG_DIR):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {"rank": rank}
    try:
        from ured_hip import syncbn
        syncbn.enable()
        assert syncbn.active()
        x = torch.from_numpy(_rows(rank))                  # [n, sets=2, N=5]
        local = torch.stack([torch.full(x.shape[1:], float(x.shape[0]), dtype=torch.float64),
                             x.mean(0), ((x - x.mean(0)) ** 2).sum(0)], dim=1)   # [2, 3, 5]
        res["merged"] = syncbn.merge_stats(local).numpy()
        res["summed"] = syncbn.sum_over_ranks(local).numpy()
        res["local_kept"] = bool(torch.equal(local[:, 0], torch.full((2, 5), float(x.shape[0]), dtype=torch.float64)))
        syncbn.disable()
        assert not syncbn.active()
    except Exception as e:
        res["error"] = repr(e)
    finally:
        q.put(res)
        dist.destroy_process_group()


def test_merge_stats_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs], key=lambda r: r["rank"])
    for p in procs:
        p.join(timeout=30)
    for r in res:
        assert "error" not in r, r
        assert r["local_kept"]
    allx = np.concatenate([_rows(0), _rows(1)])
    exp = np.stack([np.full((2, 5), allx.shape[0], np.float64), allx.mean(0), ((allx - allx.mean(0)) ** 2).sum(0)],
                   axis=1)
    np.testing.assert_allclose(res[0]["merged"], exp, rtol=1e-12, atol=1e-12)
    assert np.array_equal(res[0]["merged"], res[1]["merged"])      # the same arithmetic on every rank
    assert np.array_equal(res[0]["summed"], res[1]["summed"])
    assert res[0]["summed"][0, 0, 0] == allx.shape[0]
