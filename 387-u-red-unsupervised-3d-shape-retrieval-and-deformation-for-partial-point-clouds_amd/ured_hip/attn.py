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
_lib.register({
    "ured_attn_fwd": [_P, _I, _P, _I, _P, _I, _I, _I, _I, _I, _I, _F, _P, _I, _P, _P],
    "ured_attn_bwd": [_P, _I, _P, _I, _P, _I, _P, _P, _I, _I, _I, _I, _I, _I, _F, _P, _I, _P, _I, _P, _I, _P],
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


def self_attention(qkv, heads):
    return SelfAttnFn.apply(qkv, heads)


def cross_attention(q, kv, heads):
    return CrossAttnFn.apply(q, kv, heads)
