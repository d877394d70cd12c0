"""Graph-node multi-head softmax attention on libured_hip.so (ured_attn_fwd / ured_attn_bwd).

Node-major tensors [B, nodes, C], C = heads * d. SelfAttnFn takes the fused q|k|v
projection [B, n, 3C] of one node set; CrossAttnFn takes q [B, n, C] and the fused k|v
projection [B, m, 2C] of the other set. Both return [B, n, C] and hand back gradients in
the same fused layouts (the kernel writes the column slices in place: no split / cat).
Reference: attention_graph/attention.py:8-19 (softmax_attention) as used by
attention_gnn.py:20-32 (MultiheadAttention).
"""
import ctypes

import torch
from torch.autograd import Function

from . import _lib

_P, _I, _F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float


class UredAttnSet(ctypes.Structure):
    """include/ured_hip.h UredAttnSet: one attention call of a multi-set launch."""
    _fields_ = [("q", _P), ("ldq", _I), ("k", _P), ("ldk", _I), ("v", _P), ("ldv", _I),
                ("B", _I), ("H", _I), ("n", _I), ("m", _I), ("d", _I), ("scale", _F),
                ("out", _P), ("ldo", _I), ("weights", _P), ("dout", _P), ("lddo", _I),
                ("dq", _P), ("lddq", _I), ("dk", _P), ("lddk", _I), ("dv", _P), ("lddv", _I)]


_lib.register({
    "ured_attn_fwd": [_P, _I, _P, _I, _P, _I, _I, _I, _I, _I, _I, _F, _P, _I, _P, _P],
    "ured_attn_bwd": [_P, _I, _P, _I, _P, _I, _P, _P, _I, _I, _I, _I, _I, _I, _F, _P, _I, _P, _I, _P, _I, _P],
    "ured_attn_fwd_sets": [_I, _P, _P],
    "ured_attn_bwd_sets": [_I, _P, _P],
})


def _addr(t, col=0):
    return t.data_ptr() + 4 * col


def _fwd(qb, qcol, kb, kcol, vb, vcol, B, H, n, m, d):
    _lib.require_device(qb, kb, vb)
    out = torch.empty(B, n, H * d, device=qb.device)
    w = torch.empty(B, H, n, m, device=qb.device)
    _lib.call("ured_attn_fwd", _addr(qb, qcol), qb.shape[-1], _addr(kb, kcol), kb.shape[-1], _addr(vb, vcol),
              vb.shape[-1], B, H, n, m, d, float(d) ** -0.5, out.data_ptr(), H * d, w.data_ptr(),
              _lib.stream_of(out))
    return out, w


def _bwd(qb, qcol, kb, kcol, vb, vcol, w, dout, B, H, n, m, d, dqb, dkb, dvb):
    _lib.call("ured_attn_bwd", _addr(qb, qcol), qb.shape[-1], _addr(kb, kcol), kb.shape[-1], _addr(vb, vcol),
              vb.shape[-1], w.data_ptr(), dout.data_ptr(), dout.shape[-1], B, H, n, m, d, float(d) ** -0.5,
              _addr(dqb, qcol), dqb.shape[-1], _addr(dkb, kcol), dkb.shape[-1], _addr(dvb, vcol), dvb.shape[-1],
              _lib.stream_of(dout))


class SelfAttnFn(Function):
    @staticmethod
    def forward(ctx, qkv, heads):
        qkv = qkv.contiguous()
        B, n, C3 = qkv.shape
        C = C3 // 3
        d = C // heads
        out, w = _fwd(qkv, 0, qkv, C, qkv, 2 * C, B, heads, n, n, d)
        ctx.heads = heads
        ctx.save_for_backward(qkv, w)
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, w = ctx.saved_tensors
        B, n, C3 = qkv.shape
        C = C3 // 3
        d = C // ctx.heads
        dqkv = torch.empty_like(qkv)
        _bwd(qkv, 0, qkv, C, qkv, 2 * C, w, dout.contiguous(), B, ctx.heads, n, n, d, dqkv, dqkv, dqkv)
        return dqkv, None


class CrossAttnFn(Function):
    @staticmethod
    def forward(ctx, q, kv, heads):
        q, kv = q.contiguous(), kv.contiguous()
        B, n, C = q.shape
        m = kv.shape[1]
        d = C // heads
        out, w = _fwd(q, 0, kv, 0, kv, C, B, heads, n, m, d)
        ctx.heads = heads
        ctx.save_for_backward(q, kv, w)
        return out

    @staticmethod
    def backward(ctx, dout):
        q, kv, w = ctx.saved_tensors
        B, n, C = q.shape
        m = kv.shape[1]
        d = C // ctx.heads
        dq, dkv = torch.empty_like(q), torch.empty_like(kv)
        _bwd(q, 0, kv, 0, kv, C, w, dout.contiguous(), B, ctx.heads, n, m, d, dq, dkv, dkv)
        return dq, dkv, None


class SelfAttnPairFn(Function):
    """The two self-attention calls of a DescriptorsSelfAttention layer (node sets of n0 and n1
    nodes per sample, rows [0, B*n0) and [B*n0, B*(n0+n1)) of one fused q|k|v projection) in ONE
    forward and ONE backward launch (ured_attn_{fwd,bwd}_sets); the output and the gradient are
    row blocks of one buffer, so no split / cat. Bitwise the two SelfAttnFn calls."""

    @staticmethod
    def forward(ctx, qkv, B, n0, n1, heads):
        qkv = qkv.contiguous()
        R0 = B * n0
        C3 = qkv.shape[-1]
        C = C3 // 3
        d = C // heads
        out = torch.empty(qkv.shape[0], C, device=qkv.device)
        w0 = torch.empty(B * heads * n0 * n0 + B * heads * n1 * n1, device=qkv.device)
        sets = _sets(qkv, out, w0, None, B, n0, n1, heads, C, d)
        _lib.require_device(qkv)
        _lib.call("ured_attn_fwd_sets", 2, ctypes.byref(sets), _lib.stream_of(out))
        ctx.dims = (B, n0, n1, heads)
        ctx.save_for_backward(qkv, w0)
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, w0 = ctx.saved_tensors
        B, n0, n1, heads = ctx.dims
        C = qkv.shape[-1] // 3
        d = C // heads
        dqkv = torch.empty_like(qkv)
        dout = dout.contiguous()
        sets = _sets(qkv, None, w0, (dout, dqkv), B, n0, n1, heads, C, d)
        _lib.call("ured_attn_bwd_sets", 2, ctypes.byref(sets), _lib.stream_of(dout))
        return dqkv, None, None, None, None


def _sets(qkv, out, w, bwd, B, n0, n1, heads, C, d):
    """The two UredAttnSet entries of a self-attention pair: set 0 = rows [0, B*n0), set 1 the rest."""
    arr = (UredAttnSet * 2)()
    row0 = (0, B * n0)
    wo = (0, B * heads * n0 * n0)
    ld = qkv.shape[-1]
    for i, n in enumerate((n0, n1)):
        base = qkv.data_ptr() + 4 * row0[i] * ld
        x = arr[i]
        x.q, x.ldq, x.k, x.ldk, x.v, x.ldv = base, ld, base + 4 * C, ld, base + 8 * C, ld
        x.B, x.H, x.n, x.m, x.d, x.scale = B, heads, n, n, d, float(d) ** -0.5
        x.weights = w.data_ptr() + 4 * wo[i]
        if bwd is None:
            x.out, x.ldo = out.data_ptr() + 4 * row0[i] * C, C
        else:
            dout, dqkv = bwd
            g = dqkv.data_ptr() + 4 * row0[i] * ld
            x.dout, x.lddo = dout.data_ptr() + 4 * row0[i] * C, C
            x.dq, x.lddq, x.dk, x.lddk, x.dv, x.lddv = g, ld, g + 4 * C, ld, g + 8 * C, ld
    return arr


def self_attention(qkv, heads):
    return SelfAttnFn.apply(qkv, heads)


def self_attention_pair(qkv, B, n0, n1, heads):
    """qkv [B*n0 + B*n1, 3C] (set 0's rows first) -> attention output [B*n0 + B*n1, C]."""
    return SelfAttnPairFn.apply(qkv, B, n0, n1, heads)


def cross_attention(q, kv, heads):
    return CrossAttnFn.apply(q, kv, heads)
