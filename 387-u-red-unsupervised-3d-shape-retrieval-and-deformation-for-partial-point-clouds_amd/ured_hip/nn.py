"""Nearest-neighbour (chamfer) ops on libured_hip.so, as torch autograd Functions.

Dense form  : drop-in for chamfer_3DFunction
              (Density_aware_Chamfer_Distance/utils_v2/metrics/CD/chamfer3D/dist_chamfer_3D.py:26-64).
Ragged form : one launch for a whole family of per-sample / per-part chamfer
              calls (loss/chamfer_loss.py:13-30, loss/basic_loss.py:249-265).
Distances are squared L2 (fp32); indices int32, lowest index on ties.
"""
import torch
from torch.autograd import Function

from . import _lib

# Both directions from one evaluation of every pair distance (ured_nn_fwd_ws /
# ured_nn_seg_fwd_ws). Results are bit-identical to the two-pass kernel; the switch exists
# so the tests can run both paths.
FUSED = True
# Below ~1e8 pairs a launch is latency-bound and the two-pass kernel (one launch, no
# finalize) is faster on MI355X (16x2048x2048: 30 vs 39 us); from there up the fused one
# (64x4096x4096: 1.27x, ragged 16x16384x2048: 4.3x, 4096x1024x1024: 1.15x). When every
# segment's point sets fit the two-pass kernel's whole-set LDS tile (<= 4096 points) it stays
# ahead up to ~5e8 pairs (graph-replayed, tools/chamfer_rates.py: 8x4096x4096 42 vs 63 us,
# 16x4096x4096 75 vs 89 us; 64x4096x4096 fused 218 vs 284 us).
FUSED_MIN_PAIRS = 96 << 20
FUSED_MIN_PAIRS_SMALL_SETS = 512 << 20
TWO_PASS_ALL_TILE = 4096         # NN_TILE_ALL (csrc/nn.hip)


def use_fused(nseg, max_a, max_b):
    """Whether a launch of nseg segments of at most max_a x max_b points takes the fused path."""
    pairs = nseg * max_a * max_b
    small_sets = max(max_a, max_b) <= TWO_PASS_ALL_TILE
    return FUSED and pairs >= (FUSED_MIN_PAIRS_SMALL_SETS if small_sets else FUSED_MIN_PAIRS)


def _workspace(nseg, max_a, max_b, a_total, b_total, dirs, dev):
    if not use_fused(nseg, max_a, max_b):
        return None, 0
    nbytes = _lib.query("ured_nn_fwd_workspace", nseg, max_a, max_b, a_total, b_total, dirs)
    if nbytes == 0:
        return None, 0
    return torch.empty(nbytes, dtype=torch.uint8, device=dev), nbytes


def _as_points(t, name):
    if t.dtype != torch.float32:
        raise TypeError(f"{name}: expected float32 points, got {t.dtype}")
    if t.shape[-1] != 3:
        raise ValueError(f"{name}: last dim must be 3, got shape {tuple(t.shape)}")
    return t.contiguous()


class NNDenseFunction(Function):
    """(xyz1 [b,n,3], xyz2 [b,m,3]) -> (dist1 [b,n], dist2 [b,m], idx1 [b,n] i32, idx2 [b,m] i32)."""

    @staticmethod
    def forward(ctx, xyz1, xyz2):
        xyz1 = _as_points(xyz1, "xyz1")
        xyz2 = _as_points(xyz2, "xyz2")
        _lib.require_device(xyz1, xyz2)
        if xyz1.dim() != 3 or xyz2.dim() != 3 or xyz1.shape[0] != xyz2.shape[0]:
            raise ValueError(f"expected [b,n,3] and [b,m,3], got {tuple(xyz1.shape)} {tuple(xyz2.shape)}")
        b, n, _ = xyz1.shape
        m = xyz2.shape[1]
        dev = xyz1.device
        # dist1 / dist2 are allocations of their own, as the reference's chamfer_3DDist returns
        # them: a differentiable output that is a view made inside a custom Function rejects
        # in-place ops (dist1.clamp_()). The non-differentiable indices share one allocation.
        dist1 = torch.empty(b, n, device=dev, dtype=torch.float32)
        dist2 = torch.empty(b, m, device=dev, dtype=torch.float32)
        ibuf = torch.empty(b * (n + m), device=dev, dtype=torch.int32)
        idx1, idx2 = ibuf[:b * n].view(b, n), ibuf[b * n:].view(b, m)
        if n == 0 or m == 0:
            dist1.zero_()
            dist2.zero_()
            ibuf.zero_()
        else:
            ws, nbytes = _workspace(b, n, m, b * n, b * m, 3, dev)
            _lib.call("ured_nn_fwd_ws", _lib.ptr(xyz1), _lib.ptr(xyz2), b, n, m, 3,
                      _lib.ptr(dist1), _lib.ptr(idx1), _lib.ptr(dist2), _lib.ptr(idx2),
                      _lib.ptr(ws), nbytes, _lib.stream_of(xyz1))
        ctx.save_for_backward(xyz1, xyz2, idx1, idx2)
        ctx.mark_non_differentiable(idx1, idx2)
        return dist1, dist2, idx1, idx2

    @staticmethod
    def backward(ctx, gd1, gd2, _gi1, _gi2):
        xyz1, xyz2, idx1, idx2 = ctx.saved_tensors
        b, n, _ = xyz1.shape
        m = xyz2.shape[1]
        if not (n and m and (gd1 is not None or gd2 is not None)):
            return torch.zeros_like(xyz1), torch.zeros_like(xyz2)
        # both gradients in one allocation, every element written by the kernel (no zero fill)
        gbuf = torch.empty(3 * b * (n + m), device=xyz1.device, dtype=xyz1.dtype)
        g1, g2 = gbuf[:3 * b * n].view(b, n, 3), gbuf[3 * b * n:].view(b, m, 3)
        gd1 = gd1.contiguous() if gd1 is not None else None
        gd2 = gd2.contiguous() if gd2 is not None else None
        _lib.call("ured_nn_bwd_set", _lib.ptr(xyz1), _lib.ptr(xyz2), b, n, m,
                  _lib.ptr(gd1), _lib.ptr(gd2), _lib.ptr(idx1), _lib.ptr(idx2),
                  _lib.ptr(g1), _lib.ptr(g2), _lib.stream_of(xyz1))
        return g1, g2


class NNSegFunction(Function):
    """Ragged NN over segment pairs (see ured_nn_seg_fwd in include/ured_hip.h).

    a [Na,3], b [Nb,3] flat point buffers; segs int32 [nseg,4] device table of
    (a_off, a_len, b_off, b_len); max_a / max_b host upper bounds of the lengths.
    Returns dist_a [Na], idx_a [Na], dist_b [Nb], idx_b [Nb]; points outside every
    pair get dist 0 / idx 0 (and no gradient).
    """

    @staticmethod
    def forward(ctx, a, b, segs, max_a, max_b, dirs):
        a = _as_points(a, "a").reshape(-1, 3)
        b = _as_points(b, "b").reshape(-1, 3)
        _lib.require_device(a, b, segs)
        if segs.dtype != torch.int32 or segs.dim() != 2 or segs.shape[1] != 4:
            raise ValueError("segs must be an int32 [nseg,4] tensor")
        segs = segs.contiguous()
        dev = a.device
        # points outside every pair read 0: one zero fill for the four outputs (views of one buffer)
        Na, Nb = a.shape[0], b.shape[0]
        buf = torch.zeros(2 * (Na + Nb), device=dev, dtype=torch.float32)
        dist_a, idx_a = buf[:Na], buf[Na:2 * Na].view(torch.int32)
        dist_b, idx_b = buf[2 * Na:2 * Na + Nb], buf[2 * Na + Nb:].view(torch.int32)
        nseg = segs.shape[0]
        if nseg:
            ws, nbytes = _workspace(nseg, int(max_a), int(max_b), a.shape[0], b.shape[0], int(dirs), dev)
            _lib.call("ured_nn_seg_fwd_ws", _lib.ptr(a), _lib.ptr(b), _lib.ptr(segs), nseg,
                      int(max_a), int(max_b), int(dirs), a.shape[0], b.shape[0],
                      _lib.ptr(dist_a), _lib.ptr(idx_a), _lib.ptr(dist_b), _lib.ptr(idx_b),
                      _lib.ptr(ws), nbytes, _lib.stream_of(a))
        ctx.save_for_backward(a, b, segs, idx_a, idx_b)
        ctx.max_a, ctx.max_b, ctx.dirs = int(max_a), int(max_b), int(dirs)
        ctx.mark_non_differentiable(idx_a, idx_b)
        return dist_a, idx_a, dist_b, idx_b

    @staticmethod
    def backward(ctx, gd_a, _gia, gd_b, _gib):
        a, b, segs, idx_a, idx_b = ctx.saved_tensors
        gbuf = torch.zeros(3 * (a.shape[0] + b.shape[0]), device=a.device, dtype=a.dtype)   # one fill
        ga, gb = gbuf[:3 * a.shape[0]].view_as(a), gbuf[3 * a.shape[0]:].view_as(b)
        if not (ctx.dirs & 1):
            gd_a = None
        if not (ctx.dirs & 2):
            gd_b = None
        if segs.shape[0] and (gd_a is not None or gd_b is not None):
            gd_a = gd_a.contiguous() if gd_a is not None else None
            gd_b = gd_b.contiguous() if gd_b is not None else None
            _lib.call("ured_nn_seg_bwd", _lib.ptr(a), _lib.ptr(b), _lib.ptr(segs), segs.shape[0],
                      ctx.max_a, ctx.max_b, _lib.ptr(gd_a), _lib.ptr(gd_b),
                      _lib.ptr(idx_a), _lib.ptr(idx_b), _lib.ptr(ga), _lib.ptr(gb),
                      _lib.stream_of(a))
        return ga, gb, None, None, None, None


def nn_dense(xyz1, xyz2):
    return NNDenseFunction.apply(xyz1, xyz2)


def nn_segments(a, b, segs, max_a, max_b, dirs=3):
    """Returns dist_a, idx_a, dist_b, idx_b over the flat buffers (see NNSegFunction)."""
    a_shape, b_shape = a.shape[:-1], b.shape[:-1]
    da, ia, db, ib = NNSegFunction.apply(a.reshape(-1, 3), b.reshape(-1, 3), segs, max_a, max_b, dirs)
    return da.view(a_shape), ia.view(a_shape), db.view(b_shape), ib.view(b_shape)


DCD_MAX_POINTS = 16384


def dcd(dist1, idx1, dist2, idx2, alpha=1000.0, n_lambda=1, frac_12=None, frac_21=None):
    """Fused density-aware chamfer tail (calc_dcd, utils_v2/model_utils.py:13-51) on dense NN
    outputs: dist1/idx1 [b,n1] gt -> x, dist2/idx2 [b,n2] x -> gt (from nn_dense(gt, x)).
    Returns (loss [b], cd_p [b], cd_t [b]); forward only."""
    b, n1 = dist1.shape
    n2 = dist2.shape[1]
    frac_12 = n2 / n1 if frac_12 is None else frac_12
    frac_21 = n1 / n2 if frac_21 is None else frac_21
    _lib.require_device(dist1, dist2)
    dist1, dist2 = dist1.contiguous(), dist2.contiguous()
    idx1, idx2 = idx1.to(torch.int32).contiguous(), idx2.to(torch.int32).contiguous()
    out = torch.empty(3, b, device=dist1.device, dtype=torch.float32)
    _lib.call("ured_dcd", _lib.ptr(dist1), _lib.ptr(idx1), _lib.ptr(dist2), _lib.ptr(idx2), b, n1, n2,
              float(alpha), int(n_lambda), float(frac_12), float(frac_21),
              _lib.ptr(out[0]), _lib.ptr(out[1]), _lib.ptr(out[2]), _lib.stream_of(dist1))
    return out[0], out[1], out[2]
