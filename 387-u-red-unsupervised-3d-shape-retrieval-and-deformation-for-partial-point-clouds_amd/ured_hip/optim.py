"""FlatAdam: torch.optim.Adam (L2 weight decay, no amsgrad) with clip_grad_norm_ per module, over
flat HBM buffers (ured_adam_clip_step, csrc/optim.hip).

The reference's step tail (engine/train.py:331-346) is six clip_grad_norm_(module, 5.0) calls
and torch.optim.Adam (train_utils/optimizer_dm.py:68-104). torch's fused Adam plus the clip
walk ~500 tensors per step in multi-tensor chunks; here, at the first step, every parameter of
the six modules moves into one flat buffer (16-float aligned slices; `p.data` becomes a view of
it), with flat gradient and moment buffers beside it. Each step then gathers the step's
gradients into the flat gradient (one multi-tensor copy) and runs three launches: per-chunk fp64
sums of squares, per-module clip factors (and the per-parameter device step counters), one
float4 stream over p / g / exp_avg / exp_avg_sq.

Which parameters take a step is decided per step, as torch does: a parameter without a gradient
(`p.grad is None`: stn1/stn2/part_encoding always, re_residual_net_full until the residual loss
is switched on at epoch > init_p_m_loss) is left out of the clip norms and of Adam (no weight
decay, no moment decay, its step count does not advance). Chunks never straddle a parameter;
only the active parameters' chunks are listed, and the list is rebuilt when the set of
parameters with a gradient changes. The layout (slice order) is fixed at the first step:
the parameters active then come first, in `layout_order` if one was given (engine/dp.py passes
the order in which the first backward produced the gradients, so that its buckets fill early),
the others after them.

The gradients are gathered rather than accumulated in place: with `p.grad` kept as a view of
the flat buffer, autograd would add every new gradient into it (one extra add launch per
parameter, measured -1.2 % per step); with zero_grad(set_to_none=True) autograd hands over
fresh gradient tensors and the gather is one copy.

Semantics kept: after step() (and after gather_grads(), which engine/dp.py calls before its
all-reduce of the flat gradient) `p.grad` of every active parameter is a view of the flat
gradient and holds the clipped gradient (clip_grad_norm_ scales in place); the learning rate is
read from param_groups[0]["lr"] on every step (StepLR works unchanged) and copied to a device
scalar only when it changes (call sync_lr() before replaying a captured step after an lr
change). optimizer.state holds the flat moments and the per-parameter step counts under "flat".
"""
import ctypes
import os

import torch

from . import _lib
from .kernels import _p

_P, _I, _F, _D = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_double
_lib.register({"ured_adam_clip_step": [_P, _P, _P, _P, _P, _P, _P, _P, _I, _P, _I, _F, _P, _P, _P, _I,
                                       _D, _D, _D, _D, _P, _P, _P]})

_GRAD_VIEWS = os.environ.get("URED_GRAD_VIEWS", "1") == "1"     # A/B knob (tools/gpu_py_ab.sh)
CHUNK = 8192          # elements per workgroup (never straddles a parameter)
ALIGN = 16            # each parameter slice starts on a 64-B boundary


def _aligned(n):
    return -(-n // ALIGN) * ALIGN


def _slot_view(t):
    """(parameter, its flat-gradient view shaped like t, optimizer) or None."""
    p = t if t._base is None else t._base
    slot = getattr(p, "_ured_gslot", None)
    if not _GRAD_VIEWS or slot is None or p.numel() != t.numel() or not t.is_contiguous():
        return None
    opt, o, n = slot
    if opt.flat_grad is None:
        return None
    return p, opt.flat_grad[o:o + n].view(t.shape), opt


def grad_slot(t):
    """Output storage for the gradient of `t` — a parameter, or a same-size view of one (the
    reshaped conv weights the HIP Functions take) — inside a backward pass: (buffer, accumulate).

    When the parameter lives in a FlatAdam flat buffer and has no gradient yet, the first claim
    in a backward (one per zero_grad) gets a fresh view of its slice of the flat gradient and
    accumulate=False: the Function writes the gradient there and returns the view, autograd's
    AccumulateGrad takes it over as `p.grad` (a fresh, contiguous, layout-matching tensor is
    stolen, not copied), and gather_grads() finds it in place: no per-step copy into the flat
    buffer. A second use of the same parameter in the same backward (a layer applied twice, e.g.
    the cross-attention update of both node sets) gets the same view with accumulate=True: its
    Function adds its gradient into the view (the kernels' accumulate flag) and returns None for
    that input, so autograd has no second gradient to add: either p.grad already is the view, or
    AccumulateGrad has not run yet and will adopt (or copy) the view after this backward's kernels
    on the same stream. Every other case (no flat layout, gradients kept across backward calls, a
    double-backward) gets a fresh tensor and accumulate=False: autograd's usual accumulation.
    Contract of the accumulate path: EVERY producer of that parameter's gradient in the backward
    goes through grad_slot / grad_buffer. A non-HIP producer arriving between two HIP uses would
    make autograd sum out of place, and the later in-kernel add would land in a tensor autograd
    no longer holds; gather_grads() checks for exactly that (p.grad must be the view of an
    accumulated slot) and raises instead of losing the contribution."""
    sv = _slot_view(t)
    if sv is not None and not torch.is_grad_enabled():
        p, view, opt = sv
        if p.grad is None and getattr(p, "_ured_gclaim", None) != opt._gen:
            p._ured_gclaim = opt._gen
            return view, False
        if getattr(p, "_ured_gclaim", None) == opt._gen and (p.grad is None or p.grad.data_ptr() == view.data_ptr()):
            p._ured_gacc = opt._gen
            return view, True
    return torch.empty(t.shape, device=t.device), False


def grad_buffer(t):
    """grad_slot() for callers that cannot accumulate: the flat view on the first claim of a
    backward, else a fresh tensor (autograd accumulates)."""
    sv = _slot_view(t)
    if sv is not None and not torch.is_grad_enabled():
        p, view, opt = sv
        if p.grad is None and getattr(p, "_ured_gclaim", None) != opt._gen:
            p._ured_gclaim = opt._gen
            return view
    return torch.empty(t.shape, device=t.device)


class FlatAdam(torch.optim.Optimizer):
    def __init__(self, params, segments, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        """params: the parameters in optimizer order; segments: list of parameter lists (the
        clipping groups, one per module) covering `params` in the same order."""
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._segments = [list(s) for s in segments]
        self.flat_param = self.flat_grad = None
        self._lr_t, self._lr_host = None, None
        self._gathered = False
        self._active = None
        self._gen = 0                   # backward generation (zero_grad count), see grad_buffer()
        self.layout_order = None        # optional: parameter order for the flat layout (see module doc)

    # ---- layout -------------------------------------------------------------------------
    def _flatten(self, active_ids):
        dev = self.param_groups[0]["params"][0].device
        seen, plist, seg_of = set(), [], []
        for si, seg in enumerate(self._segments):
            for p in seg:
                if id(p) not in seen and p.requires_grad:
                    seen.add(id(p))
                    plist.append(p)
                    seg_of.append(si)
        rank = {id(p): i for i, p in enumerate(plist)}
        if self.layout_order is not None:
            pos = {id(p): i for i, p in enumerate(self.layout_order)}
            first = sorted((i for i, p in enumerate(plist) if id(p) in active_ids),
                           key=lambda i: (pos.get(id(plist[i]), len(pos)), i))
        else:
            first = [i for i, p in enumerate(plist) if id(p) in active_ids]
        rest = [i for i in range(len(plist)) if id(plist[i]) not in active_ids]
        # parameters that declare a chain (`_ured_chain`: a tuple of parameters, e.g. one
        # attention's in_proj q/k/v weights) are laid out back to back in chain order, from
        # wherever the first member falls, so that the HIP layers can use them as ONE matrix
        # (attention_graph/attention_gnn.py; ured_hip.node.fused_rows)
        seq, placed = [], set()
        for i in first + rest:
            chain = getattr(plist[i], "_ured_chain", None)
            members = [rank[id(q)] for q in chain if id(q) in rank] if chain else [i]
            cls = id(plist[i]) in active_ids
            for j in members:
                if j not in placed and (id(plist[j]) in active_ids) == cls:
                    placed.add(j)
                    seq.append(j)
        seq += [i for i in first + rest if i not in placed]
        off, total = [0] * len(plist), 0
        for i in seq:
            off[i] = total
            total += _aligned(plist[i].numel())
        self.params_all, self._seg_of, self._off, self._rank = plist, seg_of, off, rank
        self.flat_param = torch.zeros(total, device=dev)
        self.flat_grad = torch.zeros(total, device=dev)
        self.exp_avg = torch.zeros(total, device=dev)
        self.exp_avg_sq = torch.zeros(total, device=dev)
        self._gviews = []
        for p, o in zip(plist, off):
            n = p.numel()
            self.flat_param[o:o + n].copy_(p.detach().reshape(-1))
            p.data = self.flat_param[o:o + n].view_as(p)
            self._gviews.append(self.flat_grad[o:o + n].view_as(p))
            p._ured_gslot = (self, o, n)
        self._nseg = len(self._segments)
        self._coef = torch.ones(self._nseg, device=dev)
        self._lr_t = torch.zeros(1, device=dev)
        self._pstep = torch.zeros(len(plist), device=dev)
        self.state["flat"] = {"exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq, "step": self._pstep}
        self._active = None

    def _set_active(self, active):
        """Chunk tables of the parameters flagged in `active` (one bool per params_all entry),
        segment-major so that each module's chunks are contiguous."""
        dev = self.flat_param.device
        cb, ce, cs, cp, s0 = [], [], [], [], [0]
        for si in range(self._nseg):
            for i, p in enumerate(self.params_all):
                if self._seg_of[i] != si or not active[i]:
                    continue
                beg = self._off[i]
                end = beg + _aligned(p.numel())
                for b in range(beg, end, CHUNK):
                    cb.append(b)
                    ce.append(min(end, b + CHUNK))
                    cs.append(si)
                    cp.append(i)
            s0.append(len(cb))
        act = [i for i, a in enumerate(active) if a]
        self._cbeg = torch.tensor(cb or [0], dtype=torch.int64, device=dev)
        self._cend = torch.tensor(ce or [0], dtype=torch.int64, device=dev)
        self._cseg = torch.tensor(cs or [0], dtype=torch.int32, device=dev)
        self._cpar = torch.tensor(cp or [0], dtype=torch.int32, device=dev)
        self._seg0 = torch.tensor(s0, dtype=torch.int32, device=dev)
        self._act = torch.tensor(act or [0], dtype=torch.int32, device=dev)
        self._nact = len(act)
        self._nchunks = len(cb)
        self._partial = torch.zeros(max(len(cb), 1), dtype=torch.float64, device=dev)
        self._active = tuple(active)

    def active_ranges(self):
        """Flat-buffer ranges [beg, end) covering the active parameters (merged where adjacent)."""
        spans = sorted((self._off[i], self._off[i] + _aligned(p.numel()))
                       for i, p in enumerate(self.params_all) if self._active[i])
        out = []
        for b, e in spans:
            if out and out[-1][1] == b:
                out[-1][1] = e
            else:
                out.append([b, e])
        return [tuple(r) for r in out]

    def layout_key(self):
        """(offset, numel) of every parameter slice and the active flags: equal on every rank
        of a data-parallel job (engine/dp.py checks it once)."""
        return tuple((o, p.numel(), bool(a)) for o, p, a in zip(self._off, self.params_all, self._active))

    def current_active(self):
        return tuple(p.grad is not None for p in self.params_all)

    def sync_lr(self):
        lr = float(self.param_groups[0]["lr"])
        if self._lr_t is not None and lr != self._lr_host:
            self._lr_t.fill_(lr)
            self._lr_host = lr

    def prepare(self):
        """Lay out the flat buffers (first call) and refresh the chunk tables when the set of
        parameters with a gradient changed. Returns the active flags."""
        if self.flat_param is None:
            self._flatten({id(p) for s in self._segments for p in s if p.grad is not None})
        active = self.current_active()
        if active != self._active:
            self._set_active(active)
        return active

    def gather_grads(self):
        """Copy this step's gradients into the flat gradient (once per step) and point p.grad at
        their flat views. Gradients already living in their views (a captured step that keeps
        them persistent, or engine/dp.py's bucket copies) are not copied."""
        active = self.prepare()
        if self._gathered:
            return
        dst, src = [], []
        for p, v, a in zip(self.params_all, self._gviews, active):
            if not a:
                continue
            g = p.grad
            if g.data_ptr() != v.data_ptr():
                if getattr(p, "_ured_gacc", None) == self._gen:
                    raise RuntimeError("FlatAdam: a gradient accumulated in place into its flat view (grad_slot) "
                                       "was replaced by autograd (a producer outside grad_slot); it would be lost")
                dst.append(v)
                src.append(g)
            p.grad = v
        if dst:
            torch._foreach_copy_(dst, src)
        self._gathered = True

    def mark_gathered(self):
        """The caller has placed every active gradient in its flat view already."""
        for p, v, a in zip(self.params_all, self._gviews, self._active):
            if a:
                p.grad = v
        self._gathered = True

    # ---- torch.optim.Optimizer API ------------------------------------------------------
    def zero_grad(self, set_to_none=True):
        self._gathered = False
        self._gen += 1
        super().zero_grad(set_to_none=set_to_none)

    @torch.no_grad()
    def step(self, closure=None, max_norm=0.0):
        """One Adam step; max_norm > 0 first clips each module's gradient to that L2 norm."""
        loss = closure() if closure is not None else None
        self.gather_grads()
        self.sync_lr()
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        _lib.call("ured_adam_clip_step", _p(self.flat_param), _p(self.flat_grad), _p(self.exp_avg),
                  _p(self.exp_avg_sq), _p(self._cbeg), _p(self._cend), _p(self._cseg), _p(self._cpar),
                  int(self._nchunks), _p(self._seg0), int(self._nseg), float(max_norm), _p(self._lr_t),
                  _p(self._pstep), _p(self._act), int(self._nact), float(b1), float(b2), float(g["eps"]),
                  float(g["weight_decay"]), _p(self._partial), _p(self._coef), _lib.stream_of(self.flat_param))
        self._gathered = False
        return loss
