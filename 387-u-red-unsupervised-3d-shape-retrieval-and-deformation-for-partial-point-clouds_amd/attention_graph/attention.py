"""Scaled dot-product attention over graph nodes (reference attention_graph/attention.py:8-19).

query/key/value are [B, heads, head_dim, nodes]; returns (out [B, heads, head_dim, nq], weights).
"""
import torch


def softmax_attention(query, key, value):
    d = query.shape[2]
    scores = torch.einsum("bhdn,bhdm->bhnm", query, key) * d ** -0.5
    weights = scores.softmax(dim=-1)
    out = torch.einsum("bhnm,bhdm->bhdn", weights, value)
    return out, weights
