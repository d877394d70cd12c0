"""Data-parallel U-RED training: one process per GPU, gradients all-reduced over RCCL.

The reference has no distributed path (single GPU, README.md:25); the only
collective it would issue is the contrastive loss's all_gather
(loss/contrast_loss.py:35-58), which loss/contrast_loss.py keeps. This adds the
standard DP step: each rank runs the full step on its own shard of samples
(weak scaling, bs per GPU fixed), then the gradients of every trained parameter
that received one (stn1/stn2/part_encoding never do — they are skipped, the
find_unused_parameters equivalent) are averaged with bucketed all_reduce.
Buckets are flat fp32 buffers of ~bucket_mb MB, all issued asynchronously on a
communication stream once backward has finished (overlap with backward via
gradient hooks is the next step; at ~69 MB per step it is <3 % of a step).
BatchNorm uses per-rank batch statistics (what DDP does without SyncBN).
"""
import torch
import torch.distributed as dist

from engine.train import CLIPPED, TrainStep


class _Bucket:
    def __init__(self, params):
        self.params = params
        self.numel = sum(p.numel() for p in params)
        self.buf = None
        self.pending = 0
        self.work = None


class DataParallelStep(TrainStep):
    def __init__(self, cfg, db, device, bucket_mb=25.0, overlap=True):
        super().__init__(cfg, db, device)
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.overlap = overlap and self.world > 1
        # parameters in reverse registration order ~ the order backward produces their grads
        params = []
        for name in CLIPPED:
            for p in self.models[name].parameters():
                if p.requires_grad:
                    params.append(p)
        self.params = params[::-1]
        self.bucket_elems = int(bucket_mb * 1e6 / 4)
        self._buckets = None
        self._hooks = []
        self.comm_stream = torch.cuda.Stream(device=device) if self.world > 1 else None

    def _build_buckets(self):
        used = [p for p in self.params if p.grad is not None]
        buckets, cur, n = [], [], 0
        for p in used:
            cur.append(p)
            n += p.numel()
            if n >= self.bucket_elems:
                buckets.append(_Bucket(cur))
                cur, n = [], 0
        if cur:
            buckets.append(_Bucket(cur))
        self._buckets = buckets

    def reduce_gradients(self):
        if self.world == 1:
            return
        if self._buckets is None:
            self._build_buckets()     # first step: learn which parameters receive gradients
        main = torch.cuda.current_stream()
        self.comm_stream.wait_stream(main)
        works = []
        with torch.cuda.stream(self.comm_stream):
            for b in self._buckets:
                flat = torch.cat([p.grad.reshape(-1) for p in b.params])
                works.append((b, flat, dist.all_reduce(flat, op=dist.ReduceOp.SUM, async_op=True)))
        for b, flat, w in works:
            w.wait()
        main.wait_stream(self.comm_stream)
        inv = 1.0 / self.world
        for b, flat, _ in works:
            flat.mul_(inv)
            off = 0
            for p in b.params:
                n = p.numel()
                p.grad.copy_(flat[off:off + n].view_as(p.grad))
                off += n
            flat.record_stream(main)
