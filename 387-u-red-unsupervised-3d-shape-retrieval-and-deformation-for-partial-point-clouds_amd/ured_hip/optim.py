"""FlatAdam: torch.optim.Adam (L2 weight decay, no amsgrad) with clip_grad_norm_ per module, over
flat HBM buffers (ured_adam_clip_step, csrc/optim.hip).

The reference's step tail (engine/train.py:331-346) is six clip_grad_norm_(module, 5.0) calls
and torch.optim.Adam (train_utils/optimizer_dm.py:68-104). torch's fused Adam plus the clip
walk ~500 tensors per step in multi-tensor chunks; here, at the first step (when it is known
which parameters receive gradients — stn1/stn2/part_encoding never do, and Adam skips them),
every trained parameter moves into one flat buffer (16-float aligned slices, grouped by
module; `p.data` becomes a view of it), with flat gradient and moment buffers beside it. Each
step then gathers the step's gradients into the flat gradient (one multi-tensor copy) and
runs three launches: per-chunk fp64 sums of squares, per-module clip factors (and the device
step counter), one float4 stream over p / g / exp_avg / exp_avg_sq.

The gradients are gathered rather than accumulated in place: with `p.grad` kept as a view of
the flat buffer, autograd would add every new gradient into it (one extra add launch per
parameter, measured −1.2 % per step); with zero_grad(set_to_none=True) autograd hands over
fresh gradient tensors and the gather is one copy.

Semantics kept: after step() (and after gather_grads(), which engine/dp.py calls before its
all-reduce of the flat gradient) `p.grad` is a view of the flat gradient and holds the clipped
gradient (clip_grad_norm_ scales in place); the learning rate is read from
param_groups[0]["lr"] on every step (StepLR works unchanged) and copied to a device scalar
only when it changes (call sync_lr() before replaying a captured step after an lr change).
Parameters that never received a gradient at the first step are left untouched, as torch's
Adam does. optimizer.state holds the flat moments under "flat" (not per parameter).
"""
import ctypes

import torch

from . import _lib
from .kernels import _p

_P, _I, _F, _D = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_double
_lib.register({"ured_adam_clip_step": [_P, _P, _P, _P, _P, _P, _P, _I, _P, _I, _F, _P, _P,
                                       _D, _D, _D, _D, _P, _P, _P]})

CHUNK = 8192          # elements per workgroup (never straddles a module segment)
ALIGN = 16            # each parameter slice starts on a 64-B boundary


class FlatAdam(torch.optim.Optimizer):
    def __init__(self, params, segments, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        """params: the parameters in optimizer order; segments: list of parameter lists (the
        clipping groups, one per module) covering `params` in the same order."""
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._segments = [list(s) for s in segments]
        self.flat_param = self.flat_grad = None
        self._lr_t, self._lr_host = None, None
        self._gathered = False

    # ---- layout -------------------------------------------------------------------------
    def _flatten(self):
        dev = self.param_groups[0]["params"][0].device
        seg_params, offs, total = [], [], 0
        for seg in self._segments:
            ps = [p for p in seg if p.grad is not None]
            o = []
            for p in ps:
                o.append(total)
                total += -(-p.numel() // ALIGN) * ALIGN
            seg_params.append(ps)
            offs.append(o)
        self.flat_param = torch.zeros(total, device=dev)
        self.flat_grad = torch.zeros(total, device=dev)
        self.exp_avg = torch.zeros(total, device=dev)
        self.exp_avg_sq = torch.zeros(total, device=dev)
        cb, ce, cs, s0 = [], [], [], [0]
        self._gviews = []
        for si, (ps, o) in enumerate(zip(seg_params, offs)):
            for p, off in zip(ps, o):
                n = p.numel()
                self.flat_param[off:off + n].copy_(p.detach().reshape(-1))
                p.data = self.flat_param[off:off + n].view_as(p)
                self._gviews.append(self.flat_grad[off:off + n].view_as(p))
            if ps:
                beg, end = o[0], o[-1] + -(-ps[-1].numel() // ALIGN) * ALIGN
                for b in range(beg, end, CHUNK):
                    cb.append(b)
                    ce.append(min(end, b + CHUNK))
                    cs.append(si)
            s0.append(len(cb))
        self.flat_params_list = [p for ps in seg_params for p in ps]
        self._cbeg = torch.tensor(cb, dtype=torch.int64, device=dev)
        self._cend = torch.tensor(ce, dtype=torch.int64, device=dev)
        self._cseg = torch.tensor(cs, dtype=torch.int32, device=dev)
        self._seg0 = torch.tensor(s0, dtype=torch.int32, device=dev)
        self._nchunks, self._nseg = len(cb), len(self._segments)
        self._partial = torch.zeros(max(len(cb), 1), dtype=torch.float64, device=dev)
        self._coef = torch.ones(self._nseg, device=dev)
        self._lr_t = torch.zeros(1, device=dev)
        self._step_t = torch.zeros(1, device=dev)
        self.state["flat"] = {"exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq, "step": self._step_t}

    def sync_lr(self):
        lr = float(self.param_groups[0]["lr"])
        if self._lr_t is not None and lr != self._lr_host:
            self._lr_t.fill_(lr)
            self._lr_host = lr

    def gather_grads(self):
        """Copy this step's gradients into the flat gradient (once per step) and point p.grad at
        their flat views. Gradients already living in their views (a captured step that keeps
        them persistent) are not copied."""
        if self.flat_param is None:
            self._flatten()
        if self._gathered:
            return
        dst, src = [], []
        for p, v in zip(self.flat_params_list, self._gviews):
            g = p.grad
            if g is None:
                v.zero_()
            elif g.data_ptr() != v.data_ptr():
                dst.append(v)
                src.append(g)
            p.grad = v
        if dst:
            torch._foreach_copy_(dst, src)
        self._gathered = True

    # ---- torch.optim.Optimizer API ------------------------------------------------------
    def zero_grad(self, set_to_none=True):
        self._gathered = False
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
                  _p(self.exp_avg_sq), _p(self._cbeg), _p(self._cend), _p(self._cseg), int(self._nchunks),
                  _p(self._seg0), int(self._nseg), float(max_norm), _p(self._lr_t), _p(self._step_t),
                  float(b1), float(b2), float(g["eps"]), float(g["weight_decay"]), _p(self._partial),
                  _p(self._coef), _lib.stream_of(self.flat_param))
        self._gathered = False
        return loss
