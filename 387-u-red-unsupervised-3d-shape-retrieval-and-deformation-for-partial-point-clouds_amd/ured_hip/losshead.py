"""The U-RED step's loss head as ONE autograd Function on libured_hip.so (csrc/loss.hip).

engine/train.py:278-335 computes, after the networks, the weighted sum of
  cd_loss_full, cd_loss_part         compute_cm_loss(out, x, part_x, mask)       (chamfer_loss.py:13-30)
  contrast_loss                      compute_contrast_loss_loss(...)             (contrast_loss.py:61-102)
  ref_cd_loss_full (, _part)         compute_cm_loss(get_symmetric(out), ...)
  re_reg_loss_full, reg_loss_full    residual_retrieval_loss(x, out.detach(), ...) (basic_loss.py:249-265)
  recon_loss_full, recon_loss_src    compute_pc_consistency[_weighted]           (basic_consistency_loss.py)
(+ param_loss, regularization_loss.py:49-53, when enabled). As composed torch ops that is ~150
tiny kernels per step (means, masks, concatenations, normalisations, cross-entropy, and their
autograd nodes). LossHeadFn runs the same arithmetic as
  forward : cd prep, the two ragged NN launches (full and part families of out and of its mirror
            image in one launch each), the cd reduction, the point losses, the contrastive loss
            (norms + CE), the weighted sum — 8 to 10 launches;
  backward: the per-term upstream gradients, the NN weights, two a-side NN backward launches,
            the mirror fold, the point-loss and contrastive backward — 7 launches.
Every reduction is deterministic (fixed order, fp64 combine by the last workgroup).

Terms vector layout (slots): 0 cd_full, 1 cd_part, 2 ref_cd_full, 3 ref_cd_part, 4 re_reg_loss_full,
5 reg_loss_full, 6 recon_loss_full, 7 recon_loss_src, 8 contrast_loss, 9 param_loss.
"""
import ctypes
import math
import os

import torch
from torch.autograd import Function

from . import _lib
from .nn import _workspace

_P, _I, _F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float


class PointLossDesc(ctypes.Structure):
    _fields_ = [("B", _I), ("N", _I), ("S", _I), ("U", _I), ("NP", _I), ("R", _I),
                ("x", _P), ("out", _P), ("knn", _P), ("res", _P), ("rec", _P),
                ("recu", _P), ("ptsu", _P), ("inv", _P), ("mask", _P)]


ASSEMBLE_MAX = 16
USE_PART_BOUNDS = os.environ.get("URED_PART_BOUNDS", "1") != "0"   # A/B knob: 0 = slot bounds
_lib.register({
    "ured_cd_pair_prep": [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P],
    "ured_cd_pair_reduce": [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P],
    "ured_cd_pair_grad": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P],
    "ured_cd_pair_fold": [_P, _I, _I, _P, _P],
    "ured_point_losses_fwd": [ctypes.POINTER(PointLossDesc), _P, _P, _P, _P],
    "ured_point_losses_bwd": [ctypes.POINTER(PointLossDesc), _P, _P, _P, _P, _P],
    "ured_contrast_fwd": [_P, _P, _P, _I, _I, _I, _I, _F, _P, _P, _P, _P, _P, _P],
    "ured_contrast_bwd": [_P, _P, _P, _I, _I, _I, _I, _F, _P, _P, _P, _P, _P, _P],
    "ured_loss_assemble": [_I, _P, _P, _P, _P],
    "ured_loss_assemble_bwd": [_I, _P, _P, _P, _P],
})

SLOTS = ("cd_loss_full", "cd_loss_part", "ref_cd_loss_full", "ref_cd_loss_part", "re_reg_loss_full",
         "reg_loss_full", "recon_loss_full", "recon_loss_src", "contrast_loss", "param_loss")
NSLOT = len(SLOTS)
# engine/train.py:278-335 accumulation order (slot, weight key, extra factor)
ORDER = ((9, "use_param_loss", 1.0), (0, "use_chamfer_loss", 1.0), (1, "use_chamfer_part_loss", 1.0),
         (8, "use_contrast_loss", 1.0), (2, "use_symmetry_loss", 1.0), (4, "use_residuals_reg", 1.0),
         (5, "use_residuals_reg", 0.01), (6, "use_recon", 1.0), (7, "use_recon", 1.0))
LOGIT_SCALE32 = float(torch.tensor(math.log(1 / 0.07), dtype=torch.float32).exp())

_COUNTERS = {}


def _counter(dev, slot):
    """A persistent device uint (one per call site) that the last-arriving workgroup resets."""
    c = _COUNTERS.get(dev)
    if c is None:
        c = torch.zeros(16, dtype=torch.int32, device=dev)
        _COUNTERS[dev] = c
    return ctypes.c_void_p(c.data_ptr() + 4 * slot)


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _nn_seg(a, b, segs, max_a, max_b):
    """Raw ragged NN (both directions) without autograd: (dist_a, idx_a, dist_b, idx_b); points
    outside every segment are left unwritten (the head reads only segment points)."""
    dev = a.device
    Na, Nb = a.shape[0], b.shape[0]
    da = torch.empty(Na, device=dev)
    ia = torch.empty(Na, device=dev, dtype=torch.int32)
    db = torch.empty(Nb, device=dev)
    ib = torch.empty(Nb, device=dev, dtype=torch.int32)
    nseg = segs.shape[0]
    ws, nbytes = _workspace(nseg, int(max_a), int(max_b), Na, Nb, 3, dev)
    _lib.call("ured_nn_seg_fwd_ws", _p(a), _p(b), _p(segs), nseg, int(max_a), int(max_b), 3, Na, Nb,
              _p(da), _p(ia), _p(db), _p(ib), _p(ws), nbytes, _lib.stream_of(a))
    return da, ia, db, ib


class HeadInputs:
    """The non-differentiable side of the loss head for one batch.

    x [B,N,3] targets; parts: ured_hip.ops.PartBatch (x_sorted, off, counts, gid, k, mask);
    np_per_part: points per source part (1024); src_labels int64 [B,P] (-1: padding slot);
    ptsu [U,NP,3] points of the distinct source parts and inv int64 [B*P] (slot -> distinct part)
    for the weighted source reconstruction; cfg: the loss weights (use_* keys); gate: whether the
    residual loss is on this epoch (engine/train.py:308)."""

    def __init__(self, x, parts, np_per_part, src_labels, ptsu, inv, cfg, gate, bounds=None):
        self.x, self.parts, self.np, self.src_labels = x, parts, int(np_per_part), src_labels
        self.ptsu, self.inv, self.cfg, self.gate = ptsu, inv, cfg, bool(gate)
        self.bounds = bounds

    def nn_bounds(self, S, N):
        """(full-family a bound, part-family b bound) of the chamfer NN launches: the slot bounds
        (S deformed points, N target points) or, with the batch's host-side PartBounds, the most
        parts x points per part and the largest part (every segment lies within them)."""
        b = self.bounds
        if b is None or not USE_PART_BOUNDS:
            return S, N
        return min(S, b.k * self.np), min(N, b.count)

    def weights(self):
        """(slot order list for the forward sum, per-slot weights for the backward)."""
        cfg = self.cfg
        fwd, per_slot = [], [0.0] * NSLOT
        for slot, key, fac in ORDER:
            w = float(cfg.get(key, 0.0))
            if w <= 0.0:
                continue
            if slot in (4, 5) and not self.gate:
                continue
            if slot in (0, 1) and cfg.get("use_chamfer_loss", 0.0) <= 0.0:
                continue
            fwd.append((slot, w * fac))
            per_slot[slot] = w * fac
        return fwd, per_slot


class LossHeadFn(Function):
    """(out [B,S,3], res [B,N,3], rec [B,N,3], recu [U,NP,3], t [B,P,C], s [B,P,C], param 0-d
    or None) -> (loss_all, terms [10] (detached), knn [B,N] int32 (x -> out NN index))."""

    @staticmethod
    def forward(ctx, hi, out, res, rec, recu, t, s, param, contrast_ext):
        _lib.require_device(out, res, rec, recu, t, s)
        x, parts = hi.x.contiguous(), hi.parts
        B, S, _ = out.shape
        N = x.shape[1]
        P = parts.max_parts
        NP = hi.np
        dev = out.device
        out = out.contiguous()
        st = _lib.stream_of(out)
        T = torch.empty(NSLOT, device=dev)
        # --- chamfer families of out and of its mirror image ---
        A = torch.empty(2 * B, S, 3, device=dev)
        X2 = torch.empty(2 * B, N, 3, device=dev)
        XS2 = torch.empty(2 * B, N, 3, device=dev)
        segf = torch.empty(2 * B, 4, device=dev, dtype=torch.int32)
        segp = torch.empty(2 * B * P, 4, device=dev, dtype=torch.int32)
        k, counts, off = parts.k.contiguous(), parts.counts.contiguous(), parts.off.contiguous()
        _lib.call("ured_cd_pair_prep", _p(out), _p(x), _p(parts.x_sorted.contiguous()), _p(k), _p(counts), _p(off),
                  B, S, N, P, NP, _p(A), _p(X2), _p(XS2), _p(segf), _p(segp), st)
        Af, X2f, XS2f = A.view(-1, 3), X2.view(-1, 3), XS2.view(-1, 3)
        Sb, Nb = hi.nn_bounds(S, N)
        daf, iaf, dbf, ibf = _nn_seg(Af, X2f, segf, Sb, N)
        dap, iap, dbp, ibp = _nn_seg(Af, XS2f, segp, NP, Nb)
        ws = torch.empty(3 * 2 * B * (P + 1), device=dev)
        _lib.call("ured_cd_pair_reduce", _p(daf), _p(dbf), _p(dap), _p(dbp), _p(k), _p(counts), _p(off),
                  B, S, N, P, NP, _p(ws), _counter(dev, 0), _p(T), st)
        knn = ibf[:B * N].view(B, N)
        # --- residual + reconstruction losses ---
        mask = parts.mask.reshape(-1).float().contiguous()
        res, rec, recu = res.contiguous(), rec.contiguous(), recu.contiguous()
        d = PointLossDesc(B, N, S, recu.shape[0], NP, mask.shape[0], x.data_ptr(), out.data_ptr(), knn.data_ptr(),
                          res.data_ptr(), rec.data_ptr(), recu.data_ptr(), hi.ptsu.data_ptr(), hi.inv.data_ptr(),
                          mask.data_ptr())
        pws = torch.empty(3 * ((B * N + 255) // 256 + recu.shape[0]), device=dev)
        _lib.call("ured_point_losses_fwd", ctypes.byref(d), _p(pws), _counter(dev, 1), _p(T[4:]), st)
        # --- contrastive loss (single process: s_all is this rank's s; with several ranks the
        # caller computes it with the gathered codes and passes it in as contrast_ext) ---
        C = t.shape[-1]
        n = B * P
        tf, sf = t.reshape(n, C).contiguous(), s.reshape(n, C).contiguous()
        labels = hi.src_labels.reshape(n).contiguous()
        inv = torch.empty(2 * n, device=dev)
        lse = torch.empty(n, device=dev)
        if contrast_ext is None:
            cws = torch.empty(2 * n, device=dev)
            _lib.call("ured_contrast_fwd", _p(tf), _p(sf), _p(labels), n, n, C, 0, LOGIT_SCALE32, _p(inv), _p(lse),
                      _p(cws), _counter(dev, 2), _p(T[8:]), st)
        else:
            T[8:].copy_(contrast_ext.reshape(1))
        if param is not None:
            T[9:].copy_(param.reshape(1))
        else:
            T[9:].zero_()
        # --- the weighted sum (reference order) ---
        fwd, per_slot = hi.weights()
        if param is None and any(sl == 9 for sl, _ in fwd):
            raise ValueError("use_param_loss > 0 needs the param term")
        K = len(fwd)
        ptrs = (ctypes.c_void_p * ASSEMBLE_MAX)(*[T.data_ptr() + 4 * sl for sl, _ in fwd])
        wts = (ctypes.c_float * ASSEMBLE_MAX)(*[w for _, w in fwd])
        loss = torch.empty((), device=dev)
        if K:
            _lib.call("ured_loss_assemble", K, ptrs, wts, _p(loss), st)
        else:
            loss.zero_()
        ctx.hi, ctx.per_slot, ctx.shape = hi, per_slot, (B, S, N, P, NP, C, n)
        ctx.has_param = param is not None
        ctx.contrast_ext = contrast_ext is not None
        ctx.save_for_backward(A, X2, XS2, segf, segp, iaf, ibf, iap, ibp, knn, out, res, rec, recu, tf, sf,
                              labels, inv, lse, mask)
        ctx.mark_non_differentiable(T, knn)
        return loss, T, knn

    @staticmethod
    def backward(ctx, g_loss, _gT, _gknn):
        (A, X2, XS2, segf, segp, iaf, ibf, iap, ibp, knn, out, res, rec, recu, tf, sf, labels, inv, lse,
         mask) = ctx.saved_tensors
        hi = ctx.hi
        B, S, N, P, NP, C, n = ctx.shape
        dev = A.device
        st = _lib.stream_of(A)
        g_loss = g_loss.contiguous()
        gv = torch.empty(NSLOT, device=dev)
        wts = (ctypes.c_float * ASSEMBLE_MAX)(*ctx.per_slot)
        _lib.call("ured_loss_assemble_bwd", NSLOT, wts, _p(g_loss), _p(gv), st)
        need = ctx.needs_input_grad          # (hi, out, res, rec, recu, t, s, param, contrast_ext)
        parts = hi.parts
        k, counts = parts.k.contiguous(), parts.counts.contiguous()
        g_out = dres = drec = drecu = dt = ds = gcon = None
        gparam = gv[9].reshape(()) if ctx.has_param and need[7] else None
        if ctx.contrast_ext and need[8]:
            gcon = gv[8].reshape(())
        if need[5] or need[6]:
            dt = torch.empty(n, C, device=dev)
            ds = torch.empty(n, C, device=dev)
            _lib.call("ured_contrast_bwd", _p(tf), _p(sf), _p(labels), n, n, C, 0, LOGIT_SCALE32, _p(inv), _p(lse),
                      _p(gv[8:]), _p(dt), _p(ds), st)
            dt = dt.view(B, P, C) if need[5] else None
            ds = ds.view(B, P, C) if need[6] else None
        if need[2] or need[3] or need[4]:
            d = PointLossDesc(B, N, S, recu.shape[0], NP, mask.shape[0], hi.x.data_ptr(), out.data_ptr(),
                              knn.data_ptr(), res.data_ptr(), rec.data_ptr(), recu.data_ptr(), hi.ptsu.data_ptr(),
                              hi.inv.data_ptr(), mask.data_ptr())
            dres = torch.empty_like(res)
            drec = torch.empty_like(rec)
            drecu = torch.empty_like(recu)
            _lib.call("ured_point_losses_bwd", ctypes.byref(d), _p(gv[4:]), _p(dres), _p(drec), _p(drecu), st)
            dres, drec, drecu = (dres if need[2] else None), (drec if need[3] else None), (drecu if need[4] else None)
        if not need[1]:
            return (None, None, dres, drec, drecu, dt, ds, gparam, gcon)
        # chamfer: per-distance weights, a-side NN backward of both families, mirror fold
        gaf = torch.empty(2 * B * S, device=dev)
        gbf = torch.empty(2 * B * N, device=dev)
        gap = torch.empty(2 * B * S, device=dev)
        gbp = torch.empty(2 * B * N, device=dev)
        ga = torch.empty(2 * B * S, 3, device=dev)
        _lib.call("ured_cd_pair_grad", _p(gv), _p(k), _p(counts), _p(parts.gid.contiguous()), B, S, N, P, NP,
                  _p(gaf), _p(gbf), _p(gap), _p(gbp), _p(ga), st)
        Af, X2f, XS2f = A.view(-1, 3), X2.view(-1, 3), XS2.view(-1, 3)
        Sb, Nb = hi.nn_bounds(S, N)
        _lib.call("ured_nn_seg_bwd", _p(Af), _p(X2f), _p(segf), segf.shape[0], Sb, N, _p(gaf), _p(gbf),
                  _p(iaf), _p(ibf), _p(ga), None, st)
        _lib.call("ured_nn_seg_bwd", _p(Af), _p(XS2f), _p(segp), segp.shape[0], NP, Nb, _p(gap), _p(gbp),
                  _p(iap), _p(ibp), _p(ga), None, st)
        g_out = torch.empty(B, S, 3, device=dev)
        _lib.call("ured_cd_pair_fold", _p(ga), B, S, _p(g_out), st)
        return (None, g_out, dres, drec, drecu, dt, ds, gparam, gcon)


def loss_head(hi, out, res, rec, recu, t, s, param=None, contrast_ext=None):
    """-> (loss_all, {term: 0-d detached tensor} (the terms engine/train.py reports for this
    config), knn [B,N] int32 (the x -> out nearest-neighbour indices))."""
    # inputs whose terms are all off this step get no gradient (None, as in the reference: e.g. the
    # residual net before init_p_m_loss, engine/train.py:308), not a zero one
    _, w = hi.weights()
    if not (w[0] or w[1] or w[2]):
        out = out.detach()
    if not (w[4] or w[5]):
        res = res.detach()
    if not w[6]:
        rec = rec.detach()
    if not w[7]:
        recu = recu.detach()
    if not w[8] or contrast_ext is not None:
        t, s = t.detach(), s.detach()
    loss, T, knn = LossHeadFn.apply(hi, out, res, rec, recu, t, s, param, contrast_ext)
    cfg = hi.cfg
    on = {"cd_loss_full": cfg.get("use_chamfer_loss", 0.0) > 0, "cd_loss_part": cfg.get("use_chamfer_loss", 0.0) > 0,
          "ref_cd_loss_full": cfg.get("use_symmetry_loss", 0.0) > 0,
          "ref_cd_loss_part": cfg.get("use_symmetry_loss", 0.0) > 0,
          "re_reg_loss_full": cfg.get("use_residuals_reg", 0.0) > 0 and hi.gate,
          "reg_loss_full": cfg.get("use_residuals_reg", 0.0) > 0 and hi.gate,
          "recon_loss_full": cfg.get("use_recon", 0.0) > 0, "recon_loss_src": cfg.get("use_recon", 0.0) > 0,
          "contrast_loss": cfg.get("use_contrast_loss", 0.0) > 0, "param_loss": param is not None}
    return loss, {name: T[sl] for sl, name in enumerate(SLOTS) if on[name]}, knn
