"""Graph attention network of DeformNet_MatchingNet (reference attention_graph/attention_gnn.py:8-98).

Module/attribute names match the reference so checkpoints interchange. The graph has
2 global + MAX_NUM_PARTS part nodes per sample: tiny, launch-bound work. The U-RED step
runs it node-major (`forward_nodes`, [B, nodes, C]) on HIP kernels only: the q|k|v
projections as one node GEMM over the parameters' own back-to-back memory (ured_hip.node
NodeProjFn, csrc/node.hip), the attention core as one
kernel each way (ured_hip.attn), out_proj as a node GEMM, and the FeedForwardNet_norm update
(conv -> ReLU -> BatchNorm per node set -> conv, + residual) as two node GEMMs around one
BatchNorm kernel, the concatenation [x, message] read in place. `forward` keeps the
reference's channel-first signature for drop-in callers.
"""
import os

import torch
import torch.nn as nn

from ured_hip.attn import cross_attention, self_attention, self_attention_pair
from ured_hip.node import node_ffn, node_linear, node_proj

from . import get_attention_mechanism
from .attention import softmax_attention
from .attention_utils import FeedForwardNet_norm, conv1x1

_ATTN_PAIR = os.environ.get("URED_ATTN_PAIR", "1") == "1"     # A/B knob (tools/gpu_py_ab.sh)
_NODE_ALIAS = os.environ.get("URED_NODE_ALIAS", "1") == "1"   # A/B knob (tools/gpu_py_ab.sh)


class MultiheadAttention(nn.Module):
    def __init__(self, embed_dim, num_heads, attention="softmax"):
        super().__init__()
        self.embed_dim = embed_dim // num_heads          # per-head width (reference naming)
        self.attention_func = get_attention_mechanism(embed_dim, attention)
        self.num_heads = num_heads
        self.in_proj_q = nn.Conv1d(embed_dim, embed_dim, kernel_size=1)
        self.in_proj_k = nn.Conv1d(embed_dim, embed_dim, kernel_size=1)
        self.in_proj_v = nn.Conv1d(embed_dim, embed_dim, kernel_size=1)
        self.out_proj = nn.Conv1d(embed_dim, embed_dim, kernel_size=1)
        # FlatAdam lays these chains out back to back, so the node layers read q|k|v (and k|v) as
        # one matrix / bias vector without concatenating them (ured_hip.node.NodeProjFn)
        for name in ("weight", "bias"):
            chain = tuple(getattr(c, name) for c in (self.in_proj_q, self.in_proj_k, self.in_proj_v))
            for prm in chain:
                prm._ured_chain = chain

    def forward(self, query, key, value):
        b = query.shape[0]
        split = (b, self.num_heads, self.embed_dim, -1)
        out, att = self.attention_func(conv1x1(self.in_proj_q, query).view(split),
                                       conv1x1(self.in_proj_k, key).view(split),
                                       conv1x1(self.in_proj_v, value).view(split))
        return conv1x1(self.out_proj, out.reshape(b, self.num_heads * self.embed_dim, -1)), att

    @staticmethod
    def _w(conv):
        return conv.weight.view(conv.weight.shape[0], -1)

    def forward_nodes(self, xq, xkv=None, alias=False):
        """Node-major [B, n, C] query nodes and [B, m, C] key/value nodes (None: self-attention)
        -> message [B, n, C]. alias=True: (message, xq', xkv') where xq' [B*n, C] / xkv' [B*m, C]
        (None for self-attention) are the projection's alias outputs of its inputs (NodeProjFn):
        further consumers read those, and their gradients are added inside the projection's
        backward instead of by autograd."""
        if self.attention_func is not softmax_attention:
            raise NotImplementedError("node-major path implements the softmax attention only")
        q_, k_, v_ = self.in_proj_q, self.in_proj_k, self.in_proj_v
        B, n, C = xq.shape
        xq_a = xkv_a = None
        if xkv is None:
            r = node_proj((xq.reshape(B * n, C),), [(self._w(q_), self._w(k_), self._w(v_))],
                          [(q_.bias, k_.bias, v_.bias)], aliases=(alias,))
            qkv, xq_a = r if alias else (r, None)
            out = self_attention(qkv.view(B, n, 3 * C), self.num_heads)
        else:
            m = xkv.shape[1]
            r = node_proj((xq.reshape(B * n, C), xkv.reshape(B * m, C)),
                          [(self._w(q_),), (self._w(k_), self._w(v_))], [(q_.bias,), (k_.bias, v_.bias)],
                          aliases=(alias, alias))
            q, kv, xq_a, xkv_a = r if alias else (*r, None, None)
            out = cross_attention(q.view(B, n, C), kv.view(B, m, 2 * C), self.num_heads)
        msg = node_linear(out.reshape(B * n, C), self._w(self.out_proj), self.out_proj.bias).view(B, n, C)
        return (msg, xq_a, xkv_a) if alias else msg


class ResidualAttentionMessagePropagation(nn.Module):
    def __init__(self, embed_dim, num_heads, attention="softmax", use_offset=False, use_norm="use_bn"):
        super().__init__()
        self.use_offset = use_offset
        self.mha = MultiheadAttention(embed_dim, num_heads, attention)
        self.fc = FeedForwardNet_norm([2 * embed_dim, 2 * embed_dim, embed_dim], use_norm=use_norm)

    def forward(self, desc_q, desc_kv):
        message, _ = self.mha(desc_q, desc_kv, desc_kv)
        first = desc_q - message if self.use_offset else desc_q
        return desc_q + self.fc(torch.cat([first, message], dim=1))

    def forward_nodes(self, xq, xkv=None):
        return self.forward_nodes_alias(xq, xkv)[0]

    def forward_nodes_alias(self, xq, xkv=None):
        """(forward_nodes(xq, xkv), xkv') where xkv' [B, m, C] (None without xkv) stands for xkv
        in any later use: the projection returns its inputs as alias outputs (NodeProjFn), so the
        gradients of a node tensor's several consumers (q / k|v projection, the FFN, the next call)
        are summed inside the projection backward's epilogue, not by autograd adds."""
        if not self._node_ffn_ok():
            message = self.mha.forward_nodes(xq, xkv)
            first = xq - message if self.use_offset else xq
            return xq + self.fc.forward_nodes(torch.cat([first, message], dim=-1)), xkv
        B, n, C = xq.shape
        if _NODE_ALIAS:
            message, x2, xkv_a = self.mha.forward_nodes(xq, xkv, alias=True)
            xkv_a = None if xkv_a is None else xkv_a.view(xkv.shape)
        else:
            message, x2, xkv_a = self.mha.forward_nodes(xq, xkv), xq.reshape(B * n, C), xkv
        m2 = message.reshape(B * n, C)
        first, R = (x2 - m2, x2) if self.use_offset else (x2, None)
        return node_ffn(self.fc, first, m2, R, (0, B * n)).view(B, n, C), xkv_a

    def _node_ffn_ok(self):
        return self.fc.use_norm == "use_bn" and len(self.fc) == 4

    def forward_nodes_self_pair(self, x0, x1):
        """(forward_nodes(x0), forward_nodes(x1)) — the two self-attention calls of a
        DescriptorsSelfAttention layer (shared weights) — with every node GEMM run once over
        the rows of both node sets, and both sets' attention in one launch (ured_hip.attn
        SelfAttnPairFn): the attention and the BatchNorm still see one set at a time (per-set
        batch statistics, running stats updated set 0 then set 1), so the values are those of the
        two calls; half the launches, no gradient accumulation across calls."""
        mha = self.mha
        if mha.attention_func is not softmax_attention or not self._node_ffn_ok():
            return self.forward_nodes(x0), self.forward_nodes(x1)
        B, n0, C = x0.shape
        n1 = x1.shape[1]
        R0, R1 = B * n0, B * n1
        X = torch.cat([x0.reshape(R0, C), x1.reshape(R1, C)])
        q_, k_, v_ = mha.in_proj_q, mha.in_proj_k, mha.in_proj_v
        # X's second consumer (the FFN) reads the projection's alias of it (NodeProjFn)
        qkv = node_proj((X,), [(mha._w(q_), mha._w(k_), mha._w(v_))], [(q_.bias, k_.bias, v_.bias)],
                        aliases=(_NODE_ALIAS,))
        if _NODE_ALIAS:
            qkv, X = qkv
        if _ATTN_PAIR:
            # both sets' attention in one launch each way, reading / writing row blocks of qkv / o
            o = self_attention_pair(qkv, B, n0, n1, mha.num_heads)
        else:
            q0, q1 = qkv.split([R0, R1])
            o = torch.cat([self_attention(q0.view(B, n0, -1), mha.num_heads).reshape(R0, C),
                           self_attention(q1.view(B, n1, -1), mha.num_heads).reshape(R1, C)])
        message = node_linear(o, mha._w(mha.out_proj), mha.out_proj.bias)
        first, R = (X - message, X) if self.use_offset else (X, None)
        out0, out1 = node_ffn(self.fc, first, message, R, (0, R0, R0 + R1)).split([R0, R1])
        return out0.view(B, n0, C), out1.view(B, n1, C)


class DescriptorsSelfAttention(nn.Module):
    def __init__(self, embed_dim, num_heads, attention="softmax", use_offset=False):
        super().__init__()
        self.module = ResidualAttentionMessagePropagation(embed_dim, num_heads, attention, use_offset)

    def forward(self, desc0, desc1):
        return self.module(desc0, desc0), self.module(desc1, desc1)

    def forward_nodes(self, desc0, desc1):
        return self.module.forward_nodes_self_pair(desc0, desc1)


class DescriptorsCrossAttention(nn.Module):
    def __init__(self, embed_dim, num_heads, attention="softmax", use_offset=False):
        super().__init__()
        self.module = ResidualAttentionMessagePropagation(embed_dim, num_heads, attention, use_offset)

    def forward(self, desc0, desc1):
        desc0 = self.module(desc0, desc1)       # the updated desc0 feeds desc1's update
        return desc0, self.module(desc1, desc0)

    def forward_nodes(self, desc0, desc1):
        # the updated desc0 feeds desc1's update; each call hands back its key/value input as an
        # alias for the next use (see ResidualAttentionMessagePropagation.forward_nodes_alias)
        desc0, desc1 = self.module.forward_nodes_alias(desc0, desc1)
        desc1, desc0 = self.module.forward_nodes_alias(desc1, desc0)
        return desc0, desc1


class GraphAttentionNet(nn.Module):
    def __init__(self, num_stages, embed_dim, num_heads, attention="softmax", use_offset=False):
        super().__init__()
        self.layers = nn.ModuleList()
        for _ in range(num_stages):
            self.layers.append(DescriptorsSelfAttention(embed_dim, num_heads, attention, use_offset))
            self.layers.append(DescriptorsCrossAttention(embed_dim, num_heads, attention, use_offset))

    def forward(self, desc0, desc1):
        for layer in self.layers:
            desc0, desc1 = layer(desc0, desc1)
        return desc0, desc1

    def forward_nodes(self, desc0, desc1):
        """Node-major [B, n0, C], [B, n1, C]."""
        for layer in self.layers:
            desc0, desc1 = layer.forward_nodes(desc0, desc1)
        return desc0, desc1
