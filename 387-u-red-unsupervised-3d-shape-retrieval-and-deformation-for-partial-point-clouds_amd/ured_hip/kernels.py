"""Thin typed wrappers over the MLP entry points of libured_hip.so (no autograd).

Every wrapper launches on torch's current stream of the output's device and
raises on a non-zero status. Activations are point-major [M][C] fp32 tensors.
"""
import ctypes
import os

import torch

from . import _lib, syncbn

PRO_NONE, PRO_ENC, PRO_RES = 0, 1, 2
EPI_STORE, EPI_FWD, EPI_BNBWD, EPI_SPLITK = 0, 1, 2, 3
ACT_ENC, ACT_RES, ACT_BN = 0, 1, 2      # EPI_BNBWD: Conv->BN->ReLU, Conv->ReLU->BN, Conv->BN
BM = 128

_P, _I = ctypes.c_void_p, ctypes.c_int


class GemmDesc(ctypes.Structure):
    _fields_ = [("M", _I), ("N", _I), ("K", _I),
                ("a_kmajor", _I), ("b_kmajor", _I), ("pro_a", _I), ("pro_b", _I), ("epi", _I),
                ("A", _P), ("lda", _I), ("A2", _P), ("lda2", _I), ("k1", _I),
                ("B", _P), ("ldb", _I), ("pro_s", _P), ("pro_t", _P),
                ("C", _P), ("ldc", _I), ("bias", _P), ("rowbias", _P), ("ldr", _I),
                ("gidx", _P), ("group_rows", _I), ("stat_relu", _I), ("stat_ws", _P), ("pool_ws", _P),
                ("Yp", _P), ("ldy", _I), ("bn_mean", _P), ("bn_invstd", _P), ("bn_scale", _P), ("bn_shift", _P),
                ("bwd_res", _I), ("pool_idx", _P), ("pool_grad", _P), ("pool_group_rows", _I),
                ("bwd_ws", _P), ("splits", _I), ("gadd", _P), ("ldg", _I)]


_SIGS = {
    "ured_gemm": [ctypes.POINTER(GemmDesc), _P],
    "ured_splitk_reduce": [_P, _I, _I, _I, _P, _I, _I, _P, _P],
    "ured_wgrad_skinny": [_P, _I, _P, _I, _I, _I, _I, _I, _P, _P, _P, _I, _I, _P, _P],
    "ured_bn_fwd_finalize": [_P, _I, _I, _P, _P, ctypes.c_float, ctypes.c_float, _P, _P, _P, _P, _P, _P, _P, _I, _P, _P],
    "ured_bn_bwd_finalize": [_P, _I, _I, _P, _P, _P, _P, _I, _P, _P, _P, _P, _I, _P],
    "ured_bn_bwd_apply": [_P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _I, _P],
    "ured_pool_finalize": [_P, _I, _I, _I, _P, _P, _I, _P, _P, _P],
    "ured_group_colsum": [_P, _I, _I, _P, _I, _I, _P, _I, _P],
    "ured_group_colsum_split": [_P, _I, _I, _P, _I, _I, _I, _P, _P, _I, _P],
    "ured_pool_rows": [_P, _I, _I, _I, _P, _P, _I, _P, _P, _P],
    "ured_bn_act": [_P, _I, _I, _I, _P, _P, _I, _P, _I, _P],
}
_lib.register(_SIGS)


def _p(t):
    return None if t is None else t.data_ptr()


def _addr(t, elem_offset=0):
    return None if t is None else t.data_ptr() + 4 * elem_offset


def nblocks(M):
    return (M + BM - 1) // BM


_SHAPE_LOG = [] if os.environ.get("URED_GEMM_SHAPES") else None    # diagnostics: every launch's shape


# K slice per split of the few-tile store GEMMs (the per-sample fc layers, M = batch): the
# per-split K-loop is a chain of dependent DMA round trips, so shorter slices = more workgroups
_SPLITK_KMIN = 32
_SPLITK_MIN_K = 256     # split from K = 256 (the decoders' 16/256-row code gradients: 22 -> ~8 us; +0.2 % step)


def gemm(M, N, K, A, lda, B, ldb, C, ldc, *, a_kmajor=False, b_kmajor=False, pro_a=PRO_NONE, pro_b=PRO_NONE,
         epi=EPI_STORE, A_off=0, B_off=0, C_off=0, A2=None, lda2=0, k1=None, pro_s=None, pro_t=None, bias=None,
         rowbias=None, ldr=0, gidx=None, group_rows=0, stat_relu=False, stat_ws=None, pool_ws=None,
         Yp=None, ldy=0, bn=None, bwd_res=False, pool_idx=None, pool_grad=None, pool_group_rows=0,
         bwd_ws=None, splits=1, gadd=None, ldg=0):
    """One ured_gemm launch (two when a plain store GEMM with few output tiles and a long K is
    split over K: split-K partials + a reduce that adds the bias). Offsets are in elements."""
    if (epi == EPI_STORE and pro_a == PRO_NONE and pro_b == PRO_NONE and A2 is None and not a_kmajor
            and K >= _SPLITK_MIN_K):
        tiles = ((M + BM - 1) // BM) * ((N + BM - 1) // BM)
        if tiles <= 16:
            sp = min(1024 // tiles, K // _SPLITK_KMIN)
            ws = torch.empty(sp, M, N, device=C.device)
            gemm(M, N, K, A, lda, B, ldb, ws, N, b_kmajor=b_kmajor, epi=EPI_SPLITK, splits=sp,
                 A_off=A_off, B_off=B_off)
            splitk_reduce(ws, sp, M, N, C, ldc, False, C_off, bias=bias)
            return
    if _SHAPE_LOG is not None:
        _SHAPE_LOG.append((int(M), int(N), int(K), bool(a_kmajor), bool(b_kmajor), pro_a, pro_b, epi, int(splits)))
    d = GemmDesc()
    d.M, d.N, d.K = int(M), int(N), int(K)
    d.a_kmajor, d.b_kmajor, d.pro_a, d.pro_b, d.epi = int(a_kmajor), int(b_kmajor), pro_a, pro_b, epi
    d.A, d.lda = _addr(A, A_off), int(lda)
    d.A2, d.lda2, d.k1 = _p(A2), int(lda2), int(K if k1 is None else k1)
    d.B, d.ldb = _addr(B, B_off), int(ldb)
    d.pro_s, d.pro_t = _p(pro_s), _p(pro_t)
    d.C, d.ldc = _addr(C, C_off), int(ldc)
    d.bias, d.rowbias, d.ldr = _p(bias), _p(rowbias), int(ldr)
    d.gidx, d.group_rows, d.stat_relu = _p(gidx), int(group_rows), int(bool(stat_relu))
    d.stat_ws, d.pool_ws = _p(stat_ws), _p(pool_ws)
    d.Yp, d.ldy = _p(Yp), int(ldy)
    if bn is not None:
        d.bn_mean, d.bn_invstd, d.bn_scale, d.bn_shift = _p(bn.mean), _p(bn.invstd), _p(bn.scale), _p(bn.shift)
    d.bwd_res = int(bwd_res)     # ACT_ENC (False) / ACT_RES (True) / ACT_BN
    d.pool_idx, d.pool_grad, d.pool_group_rows = _p(pool_idx), _p(pool_grad), int(pool_group_rows)
    d.bwd_ws, d.splits = _p(bwd_ws), int(splits)
    d.gadd, d.ldg = _p(gadd), int(ldg)
    _lib.call("ured_gemm", ctypes.byref(d), _lib.stream_of(C))


class BNState:
    """Per-layer batch statistics of a forward pass (device vectors [N])."""
    __slots__ = ("mean", "invstd", "scale", "shift")

    def __init__(self, mean, invstd, scale, shift):
        self.mean, self.invstd, self.scale, self.shift = mean, invstd, scale, shift


class RowWeights:
    """Row multiplicities of a unique-row batch: stored row r of group r // group_rows stands
    for w[group] identical rows of the full batch (w float32 [G] on the device)."""
    __slots__ = ("w", "group_rows")

    def __init__(self, w, group_rows):
        assert group_rows % BM == 0, "row weights need whole 128-row blocks per group"
        self.w, self.group_rows = w.float().contiguous(), int(group_rows)


def _rw(rw):
    return (None, 0) if rw is None else (rw.w.data_ptr(), rw.group_rows)


def bn_fwd_finalize(stat_ws, M, N, gamma, beta, eps, momentum, running_mean, running_var, rw=None,
                    num_batches_tracked=None):
    dev = stat_ws.device
    mean = torch.empty(N, device=dev)
    invstd = torch.empty(N, device=dev)
    scale = torch.empty(N, device=dev)
    shift = torch.empty(N, device=dev)
    if syncbn.active():          # global-batch statistics over the ranks (ured_hip/syncbn.py)
        syncbn.fwd_finalize(stat_ws, M, N, gamma, beta, eps, momentum, running_mean, running_var, rw,
                            num_batches_tracked, (mean, invstd, scale, shift))
        return BNState(mean, invstd, scale, shift)
    _lib.call("ured_bn_fwd_finalize", _p(stat_ws), int(M), int(N), _p(gamma), _p(beta), float(eps), float(momentum),
              _p(running_mean), _p(running_var), _p(mean), _p(invstd), _p(scale), _p(shift), *_rw(rw),
              _p(num_batches_tracked), _lib.stream_of(stat_ws))
    return BNState(mean, invstd, scale, shift)


def bn_eval_state(gamma, beta, running_mean, running_var, eps):
    invstd = torch.rsqrt(running_var + eps)
    scale = gamma * invstd
    return BNState(running_mean.clone(), invstd, scale, beta - running_mean * scale)


def bn_bwd_finalize(bwd_ws, M, N, gamma, invstd, dgamma, dbeta, rw=None):
    dev = bwd_ws.device
    ca, cb, cc = (torch.empty(N, device=dev) for _ in range(3))
    if syncbn.active():
        syncbn.bwd_finalize(bwd_ws, M, N, gamma, invstd, dgamma, dbeta, rw, (ca, cb, cc))
        return ca, cb, cc
    _lib.call("ured_bn_bwd_finalize", _p(bwd_ws), int(M), int(N), _p(gamma), _p(invstd), _p(dgamma), _p(dbeta), 0,
              _p(ca), _p(cb), _p(cc), *_rw(rw), _lib.stream_of(bwd_ws))
    return ca, cb, cc


def bn_bwd_apply(G, Y, res, mean, coefs, want_colsum=True, rw=None):
    M, N = Y.shape
    dY = torch.empty_like(Y)
    cs = torch.empty(nblocks(M), N, device=Y.device) if want_colsum else None
    _lib.call("ured_bn_bwd_apply", _p(G), _p(Y), int(M), int(N), int(N), int(bool(res)), _p(mean),
              _p(coefs[0]), _p(coefs[1]), _p(coefs[2]), _p(dY), _p(cs), *_rw(rw), _lib.stream_of(Y))
    return dY, cs


def pool_finalize(pool_ws, M, N, group_rows, scale, shift, relu=True):
    G = M // group_rows
    pooled = torch.empty(G, N, device=pool_ws.device)
    argidx = torch.empty(G, N, device=pool_ws.device, dtype=torch.int32)
    _lib.call("ured_pool_finalize", _p(pool_ws), int(M), int(N), int(group_rows), _p(scale), _p(shift), int(relu),
              _p(pooled), _p(argidx), _lib.stream_of(pool_ws))
    return pooled, argidx


def pool_rows(Y, group_rows, scale, shift, relu=True):
    M, N = Y.shape
    G = M // group_rows
    pooled = torch.empty(G, N, device=Y.device)
    argidx = torch.empty(G, N, device=Y.device, dtype=torch.int32)
    _lib.call("ured_pool_rows", _p(Y), int(M), int(N), int(group_rows), _p(scale), _p(shift), int(relu), _p(pooled),
              _p(argidx), _lib.stream_of(Y))
    return pooled, argidx


def bn_act(Y, st, relu=True):
    """act(Y * st.scale + st.shift) materialised ([M][N])."""
    M, N = Y.shape
    out = torch.empty(M, N, device=Y.device)
    _lib.call("ured_bn_act", _p(Y), int(M), int(N), int(Y.stride(0)), _p(st.scale), _p(st.shift), int(relu),
              _p(out), int(N), _lib.stream_of(Y))
    return out


def group_colsum(X, N, G, *, off=None, group_rows=0, ldx=None, out=None, rows=None):
    """out[g] = column sums of rows [off[g], off[g+1]) (or fixed group_rows) of X[:, :N].
    Long groups are split over more workgroups (ured_group_colsum_split); `rows` = total
    rows covered (defaults to G * group_rows, or X.shape[0] for ragged groups)."""
    out = torch.empty(G, N, device=X.device) if out is None else out
    rows = (G * group_rows if off is None else X.shape[0]) if rows is None else rows
    per = max(1, rows // max(G, 1))
    blocks = ((N + 63) // 64) * G
    splits = 1
    while per // (splits * 2) >= 1024 and blocks * splits < 1024 and splits < 256:
        splits *= 2
    ws = torch.empty(G, splits, N, device=X.device) if splits > 1 else None
    _lib.call("ured_group_colsum_split", _p(X), int(N if ldx is None else ldx), int(N), _p(off), int(group_rows),
              int(G), int(splits), _p(ws), _p(out), int(out.stride(0)), _lib.stream_of(X))
    return out


def colsum(X, out=None):
    """Column sums of a [R][N] tensor (deterministic: fixed split ranges and combine order);
    into `out` [N] (contiguous) when given."""
    R, N = X.shape
    return group_colsum(X, N, 1, group_rows=R, out=None if out is None else out.view(1, N))[0]


SKINNY_WS_BLOCKS = 256          # URED_SKINNY_WS_BLOCKS (include/ured_hip.h)


def splitk_reduce(ws, splits, M, N, out, ldo, accumulate=False, out_off=0, bias=None):
    _lib.call("ured_splitk_reduce", _p(ws), int(splits), int(M), int(N), _addr(out, out_off), int(ldo),
              int(bool(accumulate)), _p(bias), _lib.stream_of(out))


_WGRAD_WGS, _WGRAD_MIN_K = 512, 512                     # swept in round 2 (choose_splits)
_WGRAD_FEW_WGS, _WGRAD_FEW_MIN_K, _WGRAD_FEW_MAX = 512, 128, 256


def choose_splits(Mo, No, K):
    """Split-K factor of a weight gradient (K = points): about 512 workgroups in total (one
    resident round of 2 blocks per CU; 1024/1536/2048 measured 0.4-1.2% slower per step), at
    least 512 points per split (128 for outputs of <= 4 tiles, whose few workgroups would
    otherwise each walk hundreds of K-steps), at most 256 splits."""
    tiles = ((Mo + 127) // 128) * ((No + 127) // 128)
    few = tiles <= 4
    min_k = _WGRAD_FEW_MIN_K if few else _WGRAD_MIN_K
    s = max(1, min((_WGRAD_FEW_WGS if few else _WGRAD_WGS) // max(tiles, 1), K // min_k))
    return max(1, min(s, _WGRAD_FEW_MAX if few else 256))


def wgrad(dY, ldd, X, ldx, Cout, Kin, Mrows, out, ldo, *, out_off=0, X_off=0, pro=PRO_NONE, pro_s=None,
          pro_t=None, accumulate=False):
    """out[cout][kin] (+)= sum_m dY[m][cout] * pro(X[m][kin]) (split-K over the Mrows points)."""
    if min(Cout, Kin) <= 4 and max(Cout, Kin) <= 256:     # 3-channel edge layers: no MFMA tile
        ws = torch.empty(SKINNY_WS_BLOCKS * Cout * Kin, device=dY.device)
        _lib.call("ured_wgrad_skinny", _p(dY), int(ldd), _addr(X, X_off), int(ldx), int(Cout), int(Kin),
                  int(Mrows), int(pro), _p(pro_s), _p(pro_t), _addr(out, out_off), int(ldo),
                  int(bool(accumulate)), _p(ws), _lib.stream_of(dY))
        return
    splits = choose_splits(Cout, Kin, Mrows)
    if splits == 1 and not accumulate:
        gemm(Cout, Kin, Mrows, dY, ldd, X, ldx, out, ldo, a_kmajor=True, b_kmajor=True, pro_b=pro,
             pro_s=pro_s, pro_t=pro_t, epi=EPI_SPLITK, splits=1, B_off=X_off, C_off=out_off)
        return
    ws = torch.empty(splits, Cout, Kin, device=dY.device)
    gemm(Cout, Kin, Mrows, dY, ldd, X, ldx, ws, Kin, a_kmajor=True, b_kmajor=True, pro_b=pro,
         pro_s=pro_s, pro_t=pro_t, epi=EPI_SPLITK, splits=splits, B_off=X_off)
    splitk_reduce(ws, splits, Cout, Kin, out, ldo, accumulate, out_off)
