"""The training step as HIP graphs (torch.cuda.CUDAGraph = hipGraph on ROCm).

An eager step issues ~1000 kernel launches (the fused HIP GEMMs plus the small torch ops of
the losses, DeformNet's projections and the optimizer) through Python, ctypes and the
autograd engine; at ~20 ms of GPU work per step that host cost is the same order as the GPU
time. The step has no host sync (segment tables, part pooling and the unique-source tables
are built on the device or from host labels before the step), so it is captured and replayed:

  graph "fwd_bwd"[key] : grads.zero_() + forward + backward (+ the data-parallel gradient
                         reduction when world > 1, see below)
  graph "update"       : clip_grad_norm_ x6 + Adam (capturable); FlatAdam reads the learning
                         rate from a device scalar, torch's optimizers get the update graph
                         re-captured when a scheduler changes the lr

key = (the batch's padded distinct-source-part count (UniqueRows with a bucket; None when the
batch encodes every slot), the residual-loss gate `epoch > init_p_m_loss`): one forward/backward
graph per key, captured the first time the key
is seen, right after that batch's step runs eagerly (so no extra optimizer step is taken and
the capture finds libraries and workspaces initialised). At most `max_graphs` are kept (LRU).
Gradients live in persistent memory, so the one update graph serves all of them: with FlatAdam
(the GPU default) the HIP layers write every gradient straight into its slice of the flat
gradient (ured_hip.optim.grad_slot), so each step starts from `p.grad = None` (no kernel) and
nothing is zeroed or added; with torch's optimizers the persistent gradient tensors are zeroed
and autograd accumulates into them. When the gate flips, the set of parameters with a gradient
changes (re_residual_net_full joins): every graph, the update graph and the persistent
gradients are dropped and the next step runs eagerly again.

Same kernels, same arithmetic as the eager step: a replay is bit-identical to an eager step on
the same state and batch.

Data parallel (world > 1): the forward contains collectives — the contrastive loss's all_gather
of the source codes and, with SyncBN, every BN layer's statistics exchange — and the backward
the bucketed gradient all-reduce (engine/dp.py FlatGradReducer: each bucket of the flat gradient
is all-reduced as soon as backward has written its last gradient). The whole reduction —
bucket all-reduces, their waits and the 1/world scaling — is part of the captured step, in one
of two forms:
  * segmented (the default at world > 1, RCCL or gloo; ured_hip/collective.py): the capture is a
    chain of graphs split at each collective. A replay runs segment 0, collective 0, segment 1, ...
    with the collectives issued eagerly on the segments' static buffers: a bucket's all_reduce is
    issued (async, on the process group's stream) right after the segment that wrote the bucket's
    last gradient and runs while the next segments — the rest of the backward — replay; the waits
    come after the last backward segment and the scaling is the last segment's tail. So only the
    last bucket's all-reduce (the last gradients backward produces; engine/dp.py keeps that
    bucket small, cfg "dp_last_bucket_mb") follows the backward. Every eager step issues the same
    bucket sequence from the same hooks, so ranks that capture at different steps still issue
    identical collective sequences. Tested at world 2 with gloo on one GPU
    (tests/test_graph_dp_gpu.py: replay == eager bitwise, bucket issue order); not yet run with
    RCCL at world > 1 (no multi-GPU box has run it).
  * inline (RCCL at world size 1 — tests/test_nccl_gpu.py — or cfg["graph_inline_collectives"]):
    the collectives are captured in the graph itself (SegmentedCapture(inline=True)), one graph,
    the bucket all-reduces on RCCL's stream inside it.
With torch's optimizers (no flat gradient) the capture holds no gradient reduction: it runs
eagerly after the replay (engine/dp.py allreduce_gradients).
"""
from collections import OrderedDict

import gc

import torch

from ured_hip.collective import SegmentedCapture
from ured_hip.ops import refresh_static


def _clone_batch(batch):
    return {k: v.clone() for k, v in batch.items()}


def _detached(T):
    """Loss dict without autograd history: a live autograd graph keeps the parameters'
    AccumulateGrad nodes (and the stream they were created on) alive, and a later capture on
    another stream would then run the gradient accumulation outside the captured graph."""
    return {k: (v.detach() if torch.is_tensor(v) else v) for k, v in T.items()}


class GraphedStep:
    def __init__(self, inner, example_batch=None, warmup=0, max_graphs=6):
        self.inner = inner
        self.max_graphs = max_graphs
        self.graphs = OrderedDict()       # key -> (static batch, graph, loss dict)
        self.g_update = None
        self.grads = None
        if warmup:                         # optional plain eager steps before the first capture
            main = torch.cuda.current_stream()
            side = torch.cuda.Stream()
            side.wait_stream(main)
            with torch.cuda.stream(side):
                for _ in range(warmup):
                    inner.step(example_batch)
            main.wait_stream(side)

    @property
    def models(self):
        return self.inner.models

    @property
    def optimizer(self):
        return self.inner.optimizer

    @property
    def scheduler(self):
        return self.inner.scheduler

    @property
    def cfg(self):
        return self.inner.cfg

    def state_dict(self):
        return self.inner.state_dict()

    def gate(self, epoch):
        cfg = self.inner.cfg
        return bool(cfg["use_residuals_reg"] > 0.0 and epoch > cfg["init_p_m_loss"])

    def key(self, batch, epoch=0):
        # the step encodes every source slot when cfg["unique_sources"] is off (engine/train.py)
        uq = batch.get("src_unique") if self.inner.cfg.get("unique_sources", True) else None
        pb = batch.get("part_bounds")          # sizes the loss head's NN launches (ured_hip/ops.py)
        return (None if uq is None else uq.U, self.gate(epoch), None if pb is None else pb.key())

    def _inline(self):
        """Capture the collectives inside the graph (RCCL) instead of splitting at them: the
        contrastive all_gather and the bucketed gradient all-reduce issued from backward's hooks,
        which then overlaps the rest of the backward on RCCL's stream within one graph.

        Only where it has run on hardware: world size 1 (tests/test_nccl_gpu.py, RCCL initialised,
        every collective captured and replayed). At world size > 1 the ranks capture at different
        steps (keys follow each rank's batches), so the inline form rests on every rank's eager
        collective sequence matching another rank's replayed one; until a multi-GPU RCCL run has
        checked averaged gradients and parameters against eager steps, world > 1 takes the
        segmented capture (collectives eagerly between graph segments, each gradient bucket's
        all-reduce issued between the backward segments) unless cfg["graph_inline_collectives"]
        asks for the inline form."""
        import torch.distributed as dist
        if not (getattr(self.inner, "collect", False) and dist.is_initialized() and dist.get_backend() == "nccl"):
            return False
        flag = self.inner.cfg.get("graph_inline_collectives")     # None: by world size; True / False: forced
        return dist.get_world_size() == 1 if flag is None else bool(flag)

    def _reduce_in_capture(self):
        """The gradient reduction is captured with the step (FlatGradReducer: every collective
        through collective.run, every tensor op on the stream); otherwise it runs after a replay."""
        return getattr(self.inner, "reducer", None) is not None

    def _flat(self):
        """FlatAdam: the HIP layers write the gradients into its persistent flat buffer."""
        return hasattr(self.inner.optimizer, "flat_grad")

    def _fresh_grads(self):
        if self._flat():
            self.inner.optimizer.zero_grad(set_to_none=True)   # the layers overwrite the flat views
        else:
            torch._foreach_zero_(self.grads)                    # keep the persistent grad tensors

    def _eager(self, batch, epoch):
        if self.grads is None:                       # first step: torch allocates the grads
            T = self.inner.step(batch, epoch)
            params = [p for m in self.inner.models.values() for p in m.parameters() if p.grad is not None]
            self.grads = [p.grad for p in params]
            return _detached(T)
        self._fresh_grads()
        loss, T = self.inner.forward(batch, epoch)
        if self._inline() or self._reduce_in_capture():
            # the same bucketed all-reduces, from the same hooks, as a replay of the captured step
            # issues (ranks can miss a graph at different steps: their collective sequences must
            # still match)
            self.inner.begin_backward()
        self.inner.backward_loss(loss)
        del loss
        self.inner.reduce_gradients()
        self.inner.clip_and_step()
        return _detached(T)

    def _capture(self, key, batch, epoch):
        self.captures = getattr(self, "captures", 0) + 1
        static = _clone_batch(batch)
        torch.cuda.synchronize()
        gc.collect()
        flat = self._flat()
        if flat:
            self.inner.optimizer.zero_grad(set_to_none=True)
        inline = self._inline()
        reduced = inline or self._reduce_in_capture()
        cap = SegmentedCapture(inline=inline)
        stream = torch.cuda.Stream()
        stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(stream):
            cap.begin()
            try:
                if not flat:
                    torch._foreach_zero_(self.grads)
                loss, T = self.inner.forward(static, epoch)
                if reduced:
                    self.inner.begin_backward()      # bucket all-reduces from the hooks
                self.inner.backward_loss(loss)
                if reduced:
                    self.inner.reduce_gradients()    # remaining buckets, waits, 1/world (flat views)
                elif flat:
                    # torch-produced gradients into their flat views, inside the captured region
                    self.inner.optimizer.gather_grads()
            except BaseException:
                cap.abort()
                raise
            cap.end()
        torch.cuda.current_stream().wait_stream(stream)
        if flat:
            opt = self.inner.optimizer
            for p, v, a in zip(opt.params_all, opt._gviews, opt._active):
                if a and p.grad.data_ptr() != v.data_ptr():
                    raise RuntimeError("graph capture: a gradient is not its flat-gradient view")
        T = _detached(T)
        del loss
        if self.g_update is None:
            self._capture_update()
        self.graphs[key] = (static, cap, T, reduced)
        while len(self.graphs) > self.max_graphs:
            self.graphs.popitem(last=False)

    def _lrs(self):
        return tuple(float(g["lr"]) for g in self.inner.optimizer.param_groups)

    def _capture_update(self):
        """The update graph: clip + optimizer step. FlatAdam reads its learning rate from a device
        scalar (sync_lr before each replay); torch's optimizers bake the float lr into the captured
        kernels, so their graph is re-captured whenever a scheduler has changed it."""
        gu = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gu):
            self.inner.clip_and_step()
        self.g_update = gu
        self._update_lrs = self._lrs()
        self.update_captures = getattr(self, "update_captures", 0) + 1

    def step(self, batch, epoch=0):
        if not self.inner.cfg.get("unique_sources", True) and "src_unique" in batch:
            # every slot encoded: the distinct-part tables are not read (and not part of the key)
            batch = {n: v for n, v in batch.items() if n != "src_unique"}
        k = self.key(batch, epoch)
        if self.grads is not None and getattr(self, "_gate", None) is not None and k[1] != self._gate:
            self.graphs.clear()          # another parameter set: re-learn the gradients eagerly
            self.g_update = None
            self.grads = None
        self._gate = k[1]
        ent = self.graphs.get(k)
        if ent is None:
            # the batch's real step runs eagerly on a side stream (that also warms up library
            # handles / workspaces for the capture stream, as capture requires), then capture
            main = torch.cuda.current_stream()
            side = torch.cuda.Stream()
            side.wait_stream(main)
            with torch.cuda.stream(side):
                T = self._eager(batch, epoch)
            main.wait_stream(side)
            self._capture(k, batch, epoch)
            return T
        self.graphs.move_to_end(k)
        static, cap, T, reduced = ent
        refresh_static(static, batch)        # one ured_copy_batch launch for the input tensors
        cap.replay()                         # segments, and the collectives between them
        if not reduced:
            self.inner.reduce_gradients()
        sync = getattr(self.inner.optimizer, "sync_lr", None)
        if sync is not None:                 # FlatAdam reads lr from a device scalar
            sync()
        elif self._lrs() != self._update_lrs:
            self._capture_update()           # lr baked into the captured kernels: re-capture
        self.g_update.replay()
        return T
