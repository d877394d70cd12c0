"""Data-parallel U-RED training: one process per GPU, gradients all-reduced over RCCL.

The reference has no distributed path (single GPU, README.md:25); the only
collective it would issue is the contrastive loss's all_gather
(loss/contrast_loss.py:35-58), which loss/contrast_loss.py keeps. This adds the
standard DP step: each rank runs the full step on its own shard of samples
(weak scaling, bs per GPU fixed), then the gradients of every trained parameter
that received one (stn1/stn2/part_encoding never do — they are skipped, the
find_unused_parameters equivalent) are averaged with bucketed all_reduce.
Buckets are flat fp32 buffers of ~bucket_mb MB, all issued asynchronously (on a
communication stream for GPU tensors) once backward has finished; at ~69 MB per
step over xGMI this is a small share of a step (overlap with backward via
gradient hooks is the next step).
BatchNorm uses per-rank batch statistics (what DDP does without SyncBN).
"""
import torch
import torch.distributed as dist

from engine.train import CLIPPED, TrainStep


def make_buckets(params, bucket_elems):
    """Group the parameters that have a gradient into ~bucket_elems-element buckets (order kept)."""
    buckets, cur, n = [], [], 0
    for p in params:
        if p.grad is None:
            continue
        cur.append(p)
        n += p.numel()
        if n >= bucket_elems:
            buckets.append(cur)
            cur, n = [], 0
    if cur:
        buckets.append(cur)
    return buckets


def allreduce_gradients(buckets, world, stream=None):
    """Average p.grad over the process group, one flat all_reduce per bucket."""
    if world == 1:
        return
    main = torch.cuda.current_stream() if stream is not None else None
    if stream is not None:
        stream.wait_stream(main)
    works = []
    ctx = torch.cuda.stream(stream) if stream is not None else _nullctx()
    with ctx:
        for b in buckets:
            flat = torch.cat([p.grad.reshape(-1) for p in b])
            works.append((b, flat, dist.all_reduce(flat, op=dist.ReduceOp.SUM, async_op=True)))
    for _, _, w in works:
        w.wait()
    if stream is not None:
        main.wait_stream(stream)
    inv = 1.0 / world
    for b, flat, _ in works:
        flat.mul_(inv)
        off = 0
        for p in b:
            n = p.numel()
            p.grad.copy_(flat[off:off + n].view_as(p.grad))
            off += n
        if stream is not None:
            flat.record_stream(main)


def allreduce_flat(flat, world, bucket_elems, stream=None):
    """Average a flat gradient buffer over the process group: all_reduce on ~bucket_elems views
    of it in place (no gather/scatter copies), all issued before the first wait."""
    main = torch.cuda.current_stream() if stream is not None else None
    if stream is not None:
        stream.wait_stream(main)
    ctx = torch.cuda.stream(stream) if stream is not None else _nullctx()
    with ctx:
        works = [dist.all_reduce(flat[o:o + bucket_elems], op=dist.ReduceOp.SUM, async_op=True)
                 for o in range(0, flat.numel(), bucket_elems)]
    for w in works:
        w.wait()
    if stream is not None:
        main.wait_stream(stream)
    flat.mul_(1.0 / world)


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class DataParallelStep(TrainStep):
    def __init__(self, cfg, db, device, bucket_mb=25.0):
        super().__init__(cfg, db, device)
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        params = []
        for name in CLIPPED:
            params += [p for p in self.models[name].parameters() if p.requires_grad]
        self.params = params[::-1]          # ~ the order backward produces gradients
        self.bucket_elems = int(bucket_mb * 1e6 / 4)
        self._buckets = None
        on_gpu = torch.device(device).type == "cuda"
        self.comm_stream = torch.cuda.Stream(device=device) if (self.world > 1 and on_gpu) else None

    def reduce_gradients(self):
        if self.world == 1:
            return
        if getattr(self.optimizer, "flat_param", None) is not None:
            # FlatAdam: gather the gradients into its flat buffer once, all-reduce that in place
            self.optimizer.gather_grads()
            allreduce_flat(self.optimizer.flat_grad, self.world, self.bucket_elems, self.comm_stream)
            return
        if self._buckets is None:           # first step: learn which parameters receive gradients
            self._buckets = make_buckets(self.params, self.bucket_elems)
        allreduce_gradients(self._buckets, self.world, self.comm_stream)
