"""Graph attention network of DeformNet_MatchingNet (reference attention_graph/attention_gnn.py:8-98).

Module/attribute names match the reference so checkpoints interchange. The
graph has 2 global + MAX_NUM_PARTS part nodes per sample: these are tiny,
latency-bound ops and stay on torch (hipBLAS) kernels.
"""
import torch
import torch.nn as nn

from . import get_attention_mechanism
from .attention_utils import FeedForwardNet_norm, conv1x1


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

    def forward(self, query, key, value):
        b = query.shape[0]
        split = (b, self.num_heads, self.embed_dim, -1)
        out, att = self.attention_func(conv1x1(self.in_proj_q, query).view(split),
                                       conv1x1(self.in_proj_k, key).view(split),
                                       conv1x1(self.in_proj_v, value).view(split))
        return conv1x1(self.out_proj, out.reshape(b, self.num_heads * self.embed_dim, -1)), att


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


class DescriptorsSelfAttention(nn.Module):
    def __init__(self, embed_dim, num_heads, attention="softmax", use_offset=False):
        super().__init__()
        self.module = ResidualAttentionMessagePropagation(embed_dim, num_heads, attention, use_offset)

    def forward(self, desc0, desc1):
        return self.module(desc0, desc0), self.module(desc1, desc1)


class DescriptorsCrossAttention(nn.Module):
    def __init__(self, embed_dim, num_heads, attention="softmax", use_offset=False):
        super().__init__()
        self.module = ResidualAttentionMessagePropagation(embed_dim, num_heads, attention, use_offset)

    def forward(self, desc0, desc1):
        desc0 = self.module(desc0, desc1)       # the updated desc0 feeds desc1's update
        return desc0, self.module(desc1, desc0)


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
