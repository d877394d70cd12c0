"""Small device-side helpers of the U-RED step (segment sums, part bookkeeping).

SegmentSumFn  : rows of x grouped into contiguous segments -> per-segment sums
                (HIP ured_group_colsum, fixed row order: deterministic).
PartBatch     : the ragged per-part view of a target batch that the reference
                builds with Python loops + torch.unique + boolean masks
                (engine/train.py:103-136): points sorted by part label, part
                offsets/counts, per-point part id, the mask of present parts.
build_parts   : computes a PartBatch with device ops only (no host sync).
"""
import ctypes

import torch
from torch.autograd import Function

from . import _lib
from . import kernels as K


class SegmentSumFn(Function):
    @staticmethod
    def forward(ctx, x, off, gid):
        x = x.contiguous()
        G = off.shape[0] - 1
        out = K.group_colsum(x, x.shape[1], G, off=off)
        ctx.save_for_backward(gid)
        return out

    @staticmethod
    def backward(ctx, gout):
        (gid,) = ctx.saved_tensors
        return gout.index_select(0, gid.long()), None, None


class GetShapeFn(Function):
    """out [J, R] = A [J, R, 6] @ p [J, 6] on HIP (ured_get_shape_fwd/bwd); gradient for p only
    (A is the source parts' data)."""

    @staticmethod
    def forward(ctx, A, p):
        if A.requires_grad:
            raise NotImplementedError("get_shape: gradients w.r.t. the source matrices are not supported")
        _lib.require_device(A, p)
        A = A.contiguous().float()
        p = p.contiguous().float()
        J, R, _ = A.shape
        out = torch.empty(J, R, device=A.device, dtype=torch.float32)
        _lib.call("ured_get_shape_fwd", _lib.ptr(A), _lib.ptr(p), J, R, _lib.ptr(out), _lib.stream_of(A))
        ctx.save_for_backward(A)
        return out

    @staticmethod
    def backward(ctx, g):
        (A,) = ctx.saved_tensors
        J, R, _ = A.shape
        gp = torch.empty(J, 6, device=A.device, dtype=torch.float32)
        _lib.call("ured_get_shape_bwd", _lib.ptr(A), _lib.ptr(g.contiguous()), J, R, _lib.ptr(gp), _lib.stream_of(A))
        return None, gp


class GetShapeSrcFn(Function):
    """get_shape(get_source_info(labels)[0], param, dflt, weight) without the gathered copy of the
    source matrices and without the mul / add / MulBackward kernels (ured_get_shape_src_fwd/bwd):
    out [J, R] with part slot j reading mats[labels[j]] (python negative indexing); gradient for
    param only (the matrices are data, dflt the parts' boxes). Bitwise the composed form."""

    @staticmethod
    def forward(ctx, mats, labels, param, dflt, weight):
        if mats.requires_grad or (dflt is not None and dflt.requires_grad):
            raise NotImplementedError("get_shape_src: gradients w.r.t. the source matrices / defaults")
        _lib.require_device(mats, labels, param)
        if mats.dtype != torch.float32 or not mats.is_contiguous() or labels.dtype != torch.int64:
            raise TypeError("get_shape_src: mats must be contiguous float32 [S, R, 6], labels int64")
        S, R, pd = mats.shape
        J = labels.numel()
        p = param.contiguous().float().reshape(J, pd)
        d = None if dflt is None else dflt.contiguous().float().reshape(J, pd)
        lab = labels.contiguous().reshape(J)
        out = torch.empty(J, R, device=mats.device, dtype=torch.float32)
        _lib.call("ured_get_shape_src_fwd", _lib.ptr(mats), _lib.ptr(lab), S, _lib.ptr(p), _lib.ptr(d), float(weight),
                  J, R, _lib.ptr(out), _lib.stream_of(mats))
        ctx.save_for_backward(mats, lab)
        ctx.weight, ctx.pshape = float(weight), param.shape
        return out

    @staticmethod
    def backward(ctx, g):
        mats, lab = ctx.saved_tensors
        S, R, _ = mats.shape
        J = lab.numel()
        gp = torch.empty(J, 6, device=mats.device, dtype=torch.float32)
        _lib.call("ured_get_shape_src_bwd", _lib.ptr(mats), _lib.ptr(lab), S, _lib.ptr(g.contiguous()), ctx.weight,
                  J, R, _lib.ptr(gp), _lib.stream_of(mats))
        return None, None, gp.view(ctx.pshape), None, None


class PermuteRowsFn(Function):
    """out[b, i] = x[b, perm[b, i]] for a per-sample permutation perm [B, N]; the backward is the
    gather by the inverse permutation (torch.gather's backward would scatter_add into zeros)."""

    @staticmethod
    def forward(ctx, x, perm, inv):
        ctx.save_for_backward(inv)
        return torch.gather(x, 1, perm.unsqueeze(-1).expand(-1, -1, x.shape[-1]))

    @staticmethod
    def backward(ctx, g):
        (inv,) = ctx.saved_tensors
        return torch.gather(g, 1, inv.unsqueeze(-1).expand(-1, -1, g.shape[-1])), None, None


def permute_rows(x, perm, inv):
    return PermuteRowsFn.apply(x, perm, inv)


class PartRowsFn(Function):
    """get_part's regrouping of per-point features (engine/train.py:103-136): x [B, N, C] ->
    (rows sorted by part label [B*N, C], per-part-slot sums [G, C]). Forward: one gather and one
    HIP segment sum; backward: ONE HIP pass (ured_part_rows_bwd) where the separate ops would
    take an index_select of the part gradients, an add and the inverse-permutation gather.

    alias=True adds a third output: x itself, for a second consumer of the features (the
    reconstruction decoder, engine/train.py:240,250). Its gradient then arrives in this backward
    beside the regrouping's and is added inside the same pass (ured_part_rows_bwd_add) instead of
    in a separate autograd add over the whole [B, N, C] tensor."""

    @staticmethod
    def forward(ctx, x, perm, inv, off, gid, alias=False):
        B, N, C = x.shape
        x = x.contiguous()
        if perm.dtype != torch.int64 or gid.dtype != torch.int32:
            raise TypeError("part_rows: perm must be int64 and gid int32")
        # the row gather xs[b*N + i] = x[b, perm[b, i]] is the backward kernel's gather with the
        # permutation in place of its inverse and no part-sum term (one float4 row copy per lane,
        # where torch.gather reads an int64 index per element)
        xs = torch.empty(B * N, C, device=x.device)
        _lib.call("ured_part_rows_bwd", _lib.ptr(x), None, _lib.ptr(perm.contiguous()), _lib.ptr(gid.contiguous()),
                  B, N, C, _lib.ptr(xs), _lib.stream_of(xs))
        sums = K.group_colsum(xs, C, off.shape[0] - 1, off=off)
        ctx.save_for_backward(inv, gid)
        ctx.shape = (B, N, C)
        return (xs, sums, x) if alias else (xs, sums)

    @staticmethod
    def backward(ctx, d_sorted, d_sums, d_x=None):
        inv, gid = ctx.saved_tensors
        B, N, C = ctx.shape
        ds = None if d_sorted is None else d_sorted.contiguous()
        dg = None if d_sums is None else d_sums.contiguous()
        dx = None if d_x is None else d_x.contiguous()
        if inv.dtype != torch.int64 or gid.dtype != torch.int32:
            raise TypeError("part_rows: inv must be int64 and gid int32")
        out = torch.empty(B, N, C, device=inv.device)
        _lib.call("ured_part_rows_bwd_add", _lib.ptr(ds), _lib.ptr(dg), _lib.ptr(inv.contiguous()),
                  _lib.ptr(gid.contiguous()), B, N, C, _lib.ptr(dx), _lib.ptr(out), _lib.stream_of(out))
        return out, None, None, None, None, None


def part_rows(x, parts, alias=False):
    """(x regrouped by part [B*N, C], per-part-slot sums [B*P, C]) for a PartBatch; alias=True
    also returns x itself as a third output whose gradient PartRowsFn adds in its own pass."""
    _lib.require_device(x)
    return PartRowsFn.apply(x, parts.perm, parts.inv_perm, parts.off, parts.gid, alias)


def segment_sum(x, off, gid):
    """x [R, C], off int32 [G+1] (row ranges), gid int32 [R] (segment of each row) -> [G, C]."""
    return SegmentSumFn.apply(x, off, gid)


class PartBatch:
    """Per-part view of a target batch.

    x_sorted [B, N, 3]  points ordered by part label (stable), i.e. the
                        reference's torch.cat over part_x[b] (engine/train.py:119,133)
    perm     [B, N]     original index of each sorted point (inv_perm: its inverse)
    gid      [B*N] i32  global part slot (b*P + rank) of each sorted point
    off      [B*P+1] i32 row offsets of each part slot in the flattened sorted rows
    counts   [B, P]     points per part slot (0 for padding slots)
    k        [B]        number of parts per sample (= mask.sum(1))
    mask     [B, P]     1 for present part slots (engine/train.py:131)
    rank_of_label [B, P] slot of each label value (valid where present)
    present  [B, P]     label value present in the sample
    """

    def __init__(self, **kw):
        self.__dict__.update(kw)

    def __len__(self):
        return self.x_sorted.shape[0]


_lib.register({"ured_build_parts": [ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_int] * 3 + [ctypes.c_void_p] * 13})


def build_parts(labels, x, max_parts, composed=None):
    """PartBatch of a target batch (engine/train.py:103-136) in ONE HIP launch (ured_build_parts:
    stable counting sort by label, slot tables, boxes and param_def); build_parts_composed is the
    same as ~20 torch ops (used for CPU tensors, or composed=True)."""
    if (not x.is_cuda) if composed is None else composed:
        return build_parts_composed(labels, x, max_parts)
    B, N = labels.shape
    P = max_parts
    dev = x.device
    lab = labels.long().contiguous()
    xf = x.float().contiguous()
    L = lambda *s: torch.empty(*s, dtype=torch.int64, device=dev)     # noqa: E731
    out = dict(x_sorted=torch.empty(B, N, 3, device=dev), perm=L(B, N), inv_perm=L(B, N),
               gid=torch.empty(B * N, dtype=torch.int32, device=dev), off=torch.empty(B * P + 1, dtype=torch.int32, device=dev),
               counts=L(B, P), k=L(B), mask=torch.empty(B, P, device=dev), rank_of_label=L(B, P),
               present=torch.empty(B, P, dtype=torch.bool, device=dev), aabb=torch.empty(B, P, 6, device=dev),
               param_def=torch.empty(B, P, 6, device=dev))
    o = out
    _lib.call("ured_build_parts", _lib.ptr(lab), _lib.ptr(xf), B, N, P, _lib.ptr(o["x_sorted"]), _lib.ptr(o["perm"]),
              _lib.ptr(o["inv_perm"]), _lib.ptr(o["gid"]), _lib.ptr(o["off"]), _lib.ptr(o["counts"]), _lib.ptr(o["k"]),
              _lib.ptr(o["mask"]), _lib.ptr(o["rank_of_label"]), _lib.ptr(o["present"]), _lib.ptr(o["aabb"]),
              _lib.ptr(o["param_def"]), _lib.stream_of(xf))
    return PartBatch(max_parts=P, **out)


def build_parts_composed(labels, x, max_parts):
    B, N = labels.shape
    P = max_parts
    dev = x.device
    lab = labels.long()
    counts_lab = torch.zeros(B, P, dtype=torch.int64, device=dev).scatter_add_(1, lab, torch.ones_like(lab))
    present = counts_lab > 0
    rank_of_label = torch.cumsum(present.long(), 1) - 1
    k = present.sum(1)
    slots = torch.arange(P, device=dev)
    mask = (slots.unsqueeze(0) < k.unsqueeze(1)).float()
    lab_sorted, perm = torch.sort(lab, dim=1, stable=True)
    inv_perm = torch.empty_like(perm).scatter_(1, perm, torch.arange(N, device=dev).expand(B, -1))
    x_sorted = torch.gather(x, 1, perm.unsqueeze(-1).expand(-1, -1, 3))
    rank_sorted = torch.gather(rank_of_label, 1, lab_sorted)
    counts = torch.zeros(B, P, dtype=torch.int64, device=dev).scatter_add_(
        1, rank_of_label.clamp(min=0), counts_lab * present)
    starts = torch.cumsum(counts, 1) - counts
    base = (torch.arange(B, device=dev) * N).unsqueeze(1)
    off = torch.cat([(base + starts).reshape(-1), torch.full((1,), B * N, device=dev, dtype=torch.int64)]).int()
    gid = (rank_sorted + (torch.arange(B, device=dev) * P).unsqueeze(1)).reshape(-1).int()
    return PartBatch(x_sorted=x_sorted, perm=perm, inv_perm=inv_perm, gid=gid, off=off, counts=counts, k=k, mask=mask,
                     rank_of_label=rank_of_label, present=present, max_parts=P)


def part_aabb(parts):
    """[B, P, 6] = (center, half extent) per part slot (compute_aabbox, dataset_utils.py:77-85):
    computed by build_parts, or one HIP segment min/max launch over the label-sorted points
    (ured_seg_aabb)."""
    if getattr(parts, "aabb", None) is not None:
        return parts.aabb
    B, N, _ = parts.x_sorted.shape
    P = parts.max_parts
    flat = parts.x_sorted.reshape(-1, 3)
    if flat.dtype != torch.float32:
        raise TypeError("part_aabb: float32 points expected")
    _lib.require_device(flat)
    flat = flat.contiguous()
    out = torch.empty(B * P, 6, device=flat.device, dtype=torch.float32)
    _lib.call("ured_seg_aabb", _lib.ptr(flat), _lib.ptr(parts.off), B * P, _lib.ptr(out), _lib.stream_of(flat))
    return out.view(B, P, 6)


class ExpandGroupsFn(Function):
    """out[r] = xu[inverse[r]] — expands the distinct rows of a unique-row batch back to the
    full batch. Backward sums the gradients of each distinct row's copies in a fixed order
    (rows sorted by `order`, segment offsets `off`; HIP group_colsum): deterministic, unlike
    index_select's atomic index_add backward."""

    @staticmethod
    def forward(ctx, xu, inverse, order, off):
        ctx.save_for_backward(order, off)
        ctx.U = xu.shape[0]
        return xu.index_select(0, inverse)

    @staticmethod
    def backward(ctx, g):
        order, off = ctx.saved_tensors
        g = g.contiguous()
        gs = g.reshape(g.shape[0], -1).index_select(0, order)
        gu = K.group_colsum(gs, gs.shape[1], ctx.U, off=off)
        return gu.view(ctx.U, *g.shape[1:]), None, None, None


def upload(a, device):
    """Host array -> device tensor. To a GPU: staged through pinned memory (torch's caching host
    allocator, which keeps the block until the copy has completed) and copied asynchronously on
    the current stream, so a per-step batch upload does not stall the host."""
    t = torch.as_tensor(a)
    if torch.device(device).type != "cuda":
        return t.to(device)
    return t.pin_memory().to(device, non_blocking=True)


class PartBounds:
    """Host-side bounds of a target batch's part structure, from the host labels (no device sync):
    k = the most parts of any target (rounded up to a multiple of 4) and count = the most points of
    any one part (rounded up to a power of two, at least 256: at most 4 x log2 distinct keys, so
    real part-size distributions do not keep evicting captured graphs). The loss head sizes its chamfer NN launches by
    them instead of by the slot bounds (P x 1024 deformed points, N target points per part): with
    the step's 4 parts per target the full family is 4096 x 2048 per target instead of 16384 x
    2048, small enough for the two-pass kernel's whole-set tile. Part of the HIP-graph key
    (engine/graph.py); rounding keeps the number of distinct keys small."""

    def __init__(self, labels_host):
        import numpy as np
        lab = np.asarray(labels_host)
        lab = lab.reshape(lab.shape[0], -1)
        k = cnt = 0
        for row in lab:
            _, c = np.unique(row, return_counts=True)
            k, cnt = max(k, int(c.shape[0])), max(cnt, int(c.max()) if c.size else 0)
        self.k = -(-k // 4) * 4
        self.count = 256
        while self.count < cnt:
            self.count *= 2

    def key(self):
        return (self.k, self.count)

    def clone(self):
        return self

    def copy_(self, other, non_blocking=False):
        assert other.key() == self.key(), "PartBounds.copy_: different bounds (part of the graph key)"
        return self


class UniqueRows:
    """Distinct entries of a batch of source-part slots (engine/train.py:196-211: every slot
    whose label is -1 — and any repeated label — encodes the same source part).

    uniq [U] (db row of each distinct part), inverse [R] (distinct part of each slot),
    order [R] (slots sorted by distinct part, stable), off int32 [U+1], w float32 [U] (copies).
    Built on the host from the host-side labels (no device sync), then copied once.
    bucket: pad U up to a multiple of `bucket` with zero-weight groups (a copy of the last
    distinct part, empty expand segment): they add nothing to the batch statistics and get
    zero gradient, and a HIP-graph step then sees a handful of distinct shapes only.
    """

    def __init__(self, labels_host, num_sources, device, bucket=None):
        import numpy as np
        s = np.asarray(labels_host).reshape(-1).astype(np.int64)
        idx = np.where(s < 0, s + num_sources, s)      # python negative indexing (dataset_utils.py:800-805)
        uniq, inv, cnt = np.unique(idx, return_inverse=True, return_counts=True)
        order = np.argsort(inv, kind="stable")
        off = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int32)
        self.U_distinct = int(uniq.shape[0])
        if bucket:
            pad = min(-(-uniq.shape[0] // bucket) * bucket, s.shape[0]) - uniq.shape[0]
            if pad > 0:
                uniq = np.concatenate([uniq, np.full(pad, uniq[-1])])
                cnt = np.concatenate([cnt, np.zeros(pad, cnt.dtype)])
                off = np.concatenate([off, np.full(pad, off[-1], np.int32)])
        self.U = int(uniq.shape[0])
        self.uniq = upload(uniq, device)
        self.inverse = upload(inv.reshape(-1).astype(np.int64), device)
        self.order = upload(order.astype(np.int64), device)
        self.off = upload(off, device)
        self.w = upload(cnt.astype(np.float32), device)

    FIELDS = ("uniq", "inverse", "order", "off", "w")

    def expand(self, xu):
        return ExpandGroupsFn.apply(xu, self.inverse, self.order, self.off)

    def clone(self):
        c = UniqueRows.__new__(UniqueRows)
        c.U, c.U_distinct = self.U, self.U_distinct
        for f in self.FIELDS:
            setattr(c, f, getattr(self, f).clone())
        return c

    def copy_(self, other, non_blocking=False):
        assert other.U == self.U, "UniqueRows.copy_: different distinct-part counts"
        for f in self.FIELDS:
            getattr(self, f).copy_(getattr(other, f), non_blocking=non_blocking)
        return self


class CopyItem(ctypes.Structure):
    _fields_ = [("dst", ctypes.c_void_p), ("src", ctypes.c_void_p), ("bytes", ctypes.c_longlong)]


COPY_MAX = 16                     # URED_COPY_MAX (include/ured_hip.h)
_lib.register({"ured_copy_batch": [ctypes.POINTER(CopyItem), ctypes.c_int, ctypes.c_void_p]})


def copy_batch(pairs):
    """dst.copy_(src) for every (dst, src) pair of same-shape, same-dtype contiguous device
    tensors, in ONE launch per 16 pairs on the current stream (ured_copy_batch) instead of one
    runtime blit each."""
    for i in range(0, len(pairs), COPY_MAX):
        part = pairs[i:i + COPY_MAX]
        arr = (CopyItem * len(part))()
        for j, (d, s) in enumerate(part):
            if d.dtype != s.dtype or d.shape != s.shape or not (d.is_contiguous() and s.is_contiguous()):
                raise ValueError(f"copy_batch: {tuple(s.shape)} {s.dtype} -> {tuple(d.shape)} {d.dtype}")
            _lib.require_device(d, s)
            arr[j].dst, arr[j].src, arr[j].bytes = d.data_ptr(), s.data_ptr(), d.numel() * d.element_size()
        _lib.call("ured_copy_batch", arr, len(part), _lib.current_stream())


def refresh_static(static, batch):
    """static[name] <- batch[name] for a captured step's input batch: tensors and the tensor
    fields of UniqueRows in one batched copy; other entries (PartBounds: host-side, part of the
    graph key) through their own copy_."""
    pairs = []
    for name, v in static.items():
        src = batch[name]
        if torch.is_tensor(v):
            pairs.append((v, src))
        elif isinstance(v, UniqueRows):
            assert src.U == v.U, "UniqueRows: different distinct-part counts"
            pairs += [(getattr(v, f), getattr(src, f)) for f in v.FIELDS]
        else:
            v.copy_(src, non_blocking=True)
    ok = [(d, s) for d, s in pairs if d.is_cuda and d.is_contiguous() and s.is_contiguous()
          and d.dtype == s.dtype and d.shape == s.shape and s.is_cuda]
    for d, s in pairs:
        if not any(d is e for e, _ in ok):
            d.copy_(s, non_blocking=True)
    copy_batch(ok)
