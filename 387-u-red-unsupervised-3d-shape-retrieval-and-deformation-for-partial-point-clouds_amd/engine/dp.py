"""Data-parallel U-RED training: one process per GPU, gradients all-reduced over RCCL.

The reference has no distributed path (single GPU, README.md:25); the only collective it would
issue is the contrastive loss's all_gather (loss/contrast_loss.py:35-58), which
loss/contrast_loss.py keeps. This adds the standard DP step: each rank runs the full step on its
own shard of samples (weak scaling, bs per GPU fixed), and the gradients of every parameter
that has one this step are averaged (stn1/stn2/part_encoding never get one and are skipped: the
find_unused_parameters equivalent; re_residual_net_full joins once the residual loss switches
on). BatchNorm uses per-rank batch statistics (what DDP does without SyncBN; cfg["sync_bn"]:
global ones, ured_hip/syncbn.py). The constructor broadcasts rank 0's parameters and buffers.

With FlatAdam (the default optimizer on the GPU) the gradients are reduced in place in its flat
gradient buffer, in buckets of ~bucket_mb MB that are issued DURING backward:
  * the first step learns the order in which backward produces the gradients (post-accumulate
    hooks) and FlatAdam lays its flat buffers out in that order, so a bucket is one contiguous
    range that fills early; the (offset, size, active) layout is checked equal on every rank
    on the first step and whenever the set of parameters with a gradient changes (an all-reduce
    of its hash), so that every rank reduces the same ranges;
  * from the second step on, each parameter's post-accumulate hook counts its bucket down;
    a full bucket's gradients are copied into their flat views (one multi-tensor copy) and its
    all_reduce is issued asynchronously (RCCL runs it on its own stream after the copy, while
    backward continues on the compute stream). Buckets are issued strictly in index order, as
    DDP does, so every rank issues the same collectives in the same order. Buckets are cut from
    the end of that order: the last one (whose all-reduce is left after the backward) is small
    (cfg "dp_last_bucket_mb", 4 MB), the others ~bucket_mb. Every collective goes through
    ured_hip/collective.run(), so a HIP-graph capture of the step (engine/graph.py) either
    captures them (RCCL, inline) or splits the captured backward at each bucket and issues the
    bucket's all-reduce between the segments of every replay, overlapping the later segments;
  * after backward: buckets that did not fill (a parameter without a gradient this step) are
    completed with zeros for the missing parameters and reduced; parameters with a gradient
    outside every bucket (one that just became active) are reduced as extra ranges; then the
    buckets are rebuilt for the new set. The flat gradient is scaled by 1/world.
Without FlatAdam (torch's Adam), `make_buckets` / `allreduce_gradients` reduce per bucket after
backward, rebuilding the buckets whenever the set of parameters with a gradient changes.
"""
import hashlib

import torch
import torch.distributed as dist

from engine.train import CLIPPED, TrainStep
from ured_hip import collective


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
    works = []
    for b in buckets:
        flat = torch.cat([p.grad.reshape(-1) for p in b])
        works.append((b, flat, dist.all_reduce(flat, op=dist.ReduceOp.SUM, async_op=True)))
    for _, _, w in works:
        w.wait()
    inv = 1.0 / world
    for b, flat, _ in works:
        flat.mul_(inv)
        off = 0
        for p in b:
            n = p.numel()
            p.grad.copy_(flat[off:off + n].view_as(p.grad))
            off += n


def allreduce_flat(flat, world, bucket_elems, ranges=None):
    """Average the given [beg, end) ranges of a flat gradient buffer over the process group:
    all_reduce on <= bucket_elems views in place, all issued before the first wait."""
    ranges = ranges or [(0, flat.numel())]
    works = []
    for b, e in ranges:
        for o in range(b, e, bucket_elems):
            works.append(dist.all_reduce(flat[o:min(e, o + bucket_elems)], op=dist.ReduceOp.SUM, async_op=True))
    for w in works:
        w.wait()
    for b, e in ranges:
        flat[b:e].mul_(1.0 / world)


def layout_hash(key):
    """A 62-bit hash of a FlatAdam layout key (identical on every rank of a correct job)."""
    return int.from_bytes(hashlib.sha256(repr(key).encode()).digest()[:8], "little") >> 2


class _Bucket:
    __slots__ = ("idx", "beg", "end", "params", "views", "pending", "launched", "work")

    def __init__(self, idx, beg, end, params, views):
        self.idx, self.beg, self.end, self.params, self.views = idx, beg, end, params, views
        self.pending, self.launched, self.work = len(params), False, None


class FlatGradReducer:
    """Bucketed all-reduce of FlatAdam's flat gradient, issued from backward's gradient hooks
    (see the module docstring). Usage per step: begin() before backward, finish() after it."""

    def __init__(self, optimizer, params, world, bucket_elems, overlap=True, last_elems=None):
        self.opt, self.world, self.bucket_elems, self.overlap = optimizer, world, bucket_elems, overlap
        self.last_elems = bucket_elems if last_elems is None else max(1, int(last_elems))
        self.issued = []                    # bucket indices in all-reduce issue order (tests clear / read it)
        self.deferred = []                  # captured hooks that ran off the capture stream (diagnostics)
        self._arrival = []                  # first step: gradient arrival order
        self._fb = None                     # buckets over the flat gradient
        self._fb_key = None
        self._bucket_of = {}
        self._next = 0
        self._armed = False
        self._step_armed = False
        self._checked = None                # the active set whose layout was last checked across ranks
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in params] if overlap else []

    # hooks run on the autograd thread, in gradient-production order
    def _on_grad(self, p):
        if not self._armed:
            if self._fb is None:
                self._arrival.append(p)
            return
        b = self._bucket_of.get(id(p))
        if b is None:
            return                        # not in a bucket: handled after backward
        b.pending -= 1
        cs = collective.capture_stream()
        if cs is not None and torch.cuda.current_stream() != cs:
            # a captured step whose hook runs on another stream than the capture's (the autograd
            # engine runs a parameter's gradient accumulation on the stream its accumulator node was
            # created on): a graph split or a copy from here would not land in the captured
            # sequence. The bucket is left to finish(), on the capture stream, in the same order.
            self.deferred.append((b.idx, int(torch.cuda.current_stream().stream_id), int(cs.stream_id)))
            return
        if b.pending == 0 and b.idx == self._next:
            fb, ready = self._fb, []
            while self._next < len(fb) and fb[self._next].pending == 0:
                self._prepare(fb[self._next])
                ready.append(fb[self._next])
                self._next += 1
            collective.run(self._issue_fn(ready))     # one host step (one graph split) per hook

    def _prepare(self, b, fill_missing=False):
        """The GPU side of a bucket before its all-reduce: gradients that are not their flat views
        (torch-produced) copied in, missing ones zeroed (after backward only). Captured into the
        current graph segment when a graph capture is running."""
        dst, src = [], []
        for p, v in zip(b.params, b.views):
            g = p.grad
            if g is None:
                if fill_missing:
                    v.zero_()
                continue
            if g.data_ptr() != v.data_ptr():
                dst.append(v)
                src.append(g)
        if dst:
            torch._foreach_copy_(dst, src)
        b.launched = True

    def _issue_fn(self, bs, wait=()):
        """The host side: all_reduce of each bucket's flat slice (async) issued in bucket order,
        then the waits of `wait`. Goes through collective.run(): eagerly it runs at once; while a
        segmented capture records the step (engine/graph.py) it closes the graph segment and runs
        between segments at every replay — after the kernels that wrote the bucket, before the
        rest of the backward, so the reduction overlaps it."""
        flat = self.opt.flat_grad
        views = [flat[b.beg:b.end] for b in bs]

        def fn():
            for b, v in zip(bs, views):
                b.work = dist.all_reduce(v, op=dist.ReduceOp.SUM, async_op=True)
                self.issued.append(b.idx)
            for b in wait:
                b.work.wait()
        return fn

    def _reduce_ranges(self, ranges):
        """Average [beg, end) ranges of the flat gradient outside the buckets: <= bucket_elems views
        all-reduced (issued, then waited, through collective.run), then scaled by 1/world."""
        flat = self.opt.flat_grad
        views = [flat[o:min(e, o + self.bucket_elems)] for b, e in ranges for o in range(b, e, self.bucket_elems)]

        def fn():
            works = [dist.all_reduce(v, op=dist.ReduceOp.SUM, async_op=True) for v in views]
            for w in works:
                w.wait()
        collective.run(fn)
        for b, e in ranges:
            flat[b:e].mul_(1.0 / self.world)

    def _build(self):
        """Buckets over the flat gradient in backward's production order, cut from the END: the
        last bucket (the last gradients backward produces, whose all-reduce is the one left
        exposed after the backward) holds ~last_elems elements, the others ~bucket_elems. A bucket
        is a contiguous range (parameters without a gradient this step split it)."""
        from ured_hip.optim import _aligned
        opt = self.opt
        slot = sorted((opt._off[i], i) for i, a in enumerate(opt._active) if a)
        groups, cur, beg, n, limit = [], [], 0, 0, self.last_elems
        for o, i in reversed(slot):
            if cur and (o + _aligned(opt.params_all[i].numel()) != beg or n >= limit):
                groups.append(cur)
                cur, n, limit = [], 0, self.bucket_elems
            cur.append(i)
            beg = o
            n += opt.params_all[i].numel()
        if cur:
            groups.append(cur)
        fb = []
        for g in reversed(groups):
            g = g[::-1]
            fb.append(_Bucket(len(fb), opt._off[g[0]], opt._off[g[-1]] + _aligned(opt.params_all[g[-1]].numel()),
                              [opt.params_all[j] for j in g], [opt._gviews[j] for j in g]))
        self._fb, self._fb_key = fb, opt._active
        self._bucket_of = {id(p): b for b in fb for p in b.params}

    def _check_layout(self):
        h = layout_hash(self.opt.layout_key())
        t = torch.tensor([h, -h], dtype=torch.int64, device=self.opt.flat_grad.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if int(t[0]) != h or -int(t[1]) != h:
            raise RuntimeError("data-parallel: the flat gradient layout differs between ranks "
                               "(different parameter sets with gradients); refusing to all-reduce")
        self._checked = self.opt._active

    @property
    def num_buckets(self):
        return 0 if self._fb is None else len(self._fb)

    def begin(self):
        """Before backward: arm the hooks (from the second step on)."""
        self._step_armed = self._fb is not None
        if self._step_armed:
            for b in self._fb:
                b.pending, b.launched, b.work = len(b.params), False, None
            self._next = 0
        self._armed = self._step_armed

    def finish(self):
        """After backward: complete the reduction; the flat gradient holds the rank average and
        p.grad of every active parameter is its flat view. Every collective goes through
        collective.run(), every tensor op stays on the stream: called inside a graph capture
        (engine/graph.py) the whole reduction is part of the captured step, its collectives either
        captured (RCCL, inline) or issued between the graph segments at every replay."""
        self._armed = False
        armed, self._step_armed = self._step_armed, False
        opt = self.opt
        if opt.flat_param is None and self._arrival:
            opt.layout_order = list(self._arrival)        # first step: backward's order
        active = opt.prepare()
        capturing = torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
        if capturing:
            # a captured finish() must not sync (the layout check reads its all-reduced hash on
            # the host) nor rebuild the buckets (their ranges are baked into the graph): the eager
            # step of the same key, which always runs before its capture, has done both
            if self._checked != active or (self.overlap and self._fb_key != active):
                raise RuntimeError("data-parallel: a layout check or bucket rebuild is pending inside a "
                                   "graph capture (run the step of this key eagerly first)")
        if self._checked != active:
            # first step, or the set of parameters with a gradient changed (e.g. the residual net
            # joining): every rank must reduce the same ranges — checked again (one tiny
            # all_reduce, only when the set changes)
            self._check_layout()
        if not armed or not any(b.launched for b in self._fb):
            # first step (overlap off, or no bucket filled during backward): all after backward
            opt.gather_grads()
            self._reduce_ranges(opt.active_ranges())
            opt.mark_gathered()
            if self.overlap and self._fb_key != active:
                self._build()
            return
        rest = self._fb[self._next:]                      # buckets that did not fill, in order
        for b in rest:
            self._prepare(b, fill_missing=True)
        extra = [i for i, a in enumerate(active) if a and id(opt.params_all[i]) not in self._bucket_of]
        if extra and capturing:
            raise RuntimeError("data-parallel: a parameter outside every bucket inside a graph capture")
        for i in extra:                                   # parameters that just became active
            opt._gviews[i].copy_(opt.params_all[i].grad)
        # the remaining buckets' all-reduces and the waits of every bucket, as one host step
        collective.run(self._issue_fn(rest, wait=self._fb))
        if extra:
            self._reduce_ranges([(opt._off[i], opt._off[i] + opt.params_all[i].numel()) for i in extra])
        for b in self._fb:
            opt.flat_grad[b.beg:b.end].mul_(1.0 / self.world)
        opt.mark_gathered()
        if self._fb_key != active:
            self._build()


class DataParallelStep(TrainStep):
    """cfg["dp_force_collectives"]: run every collective (bucketed gradient all-reduce, the
    contrastive all_gather) through the process group even at world size 1 — the test hook that
    exercises the RCCL code paths, eager and captured, on a one-GPU box."""

    def __init__(self, cfg, db, device, bucket_mb=None, overlap=None, last_bucket_mb=None):
        super().__init__(cfg, db, device)
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.collect = self.world > 1 or (bool(cfg.get("dp_force_collectives", False)) and dist.is_initialized())
        self.force_gather = self.collect     # this step's contrastive codes go through the group
        if self.world > 1:
            self.broadcast_state()
        params = []
        for name in CLIPPED:
            params += [p for p in self.models[name].parameters() if p.requires_grad]
        self.params = params[::-1]          # ~ the order backward produces gradients
        if bucket_mb is None:
            bucket_mb = cfg.get("dp_bucket_mb", 25.0)
        self.bucket_elems = int(bucket_mb * 1e6 / 4)
        self._buckets = None                # torch-Adam path: (active key, buckets)
        overlap = self.collect if overlap is None else bool(overlap)
        # the last bucket is the one whose all-reduce follows the backward: kept small (cfg
        # "dp_last_bucket_mb", default 4 MB; the others ~bucket_mb)
        last_mb = cfg.get("dp_last_bucket_mb", 4.0) if last_bucket_mb is None else last_bucket_mb
        self.reducer = (FlatGradReducer(self.optimizer, params, self.world, self.bucket_elems, overlap,
                                        last_elems=int(last_mb * 1e6 / 4))
                        if self.collect and hasattr(self.optimizer, "prepare") else None)

    def broadcast_state(self, src=0):
        """Every rank starts from rank src's parameters and buffers (as DDP's constructor does:
        each process initialised its modules from its own RNG stream)."""
        with torch.no_grad():
            for name in sorted(self.models):
                for t in list(self.models[name].parameters()) + list(self.models[name].buffers()):
                    dist.broadcast(t.data, src)

    def begin_backward(self):
        if self.reducer is not None:
            self.reducer.begin()

    def reduce_gradients(self):
        if not self.collect:
            return
        if self.reducer is not None:
            self.reducer.finish()
            return
        # torch's Adam: per-bucket reduction after backward; buckets follow the active set
        key = tuple(p.grad is not None for p in self.params)
        if self._buckets is None or self._buckets[0] != key:
            self._buckets = (key, make_buckets(self.params, self.bucket_elems))
        allreduce_gradients(self._buckets[1], self.world)
