"""Graph attention used by DeformNet_MatchingNet (reference attention_graph/__init__.py:13-33).

Only the softmax mechanism is on the U-RED path; the FAVOR / linear variants of
the reference (attention.py:22-118) are out of scope.
"""
from .attention import softmax_attention


def get_attention_mechanism(embed_dim, attention_name):
    if attention_name == "softmax":
        return softmax_attention
    raise ValueError(f"Attention type {attention_name} is not supported (only 'softmax' is on the U-RED path).")


__all__ = ["get_attention_mechanism"]
