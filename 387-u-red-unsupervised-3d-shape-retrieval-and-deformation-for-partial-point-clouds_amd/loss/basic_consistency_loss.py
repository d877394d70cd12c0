"""Drop-in for the reference loss/basic_consistency_loss.py:4-22 (reconstruction MSEs)."""
import torch


def compute_pc_consistency(pc1, pc2):
    d = pc1 - pc2
    return (d * d).sum(-1).mean()


def compute_pc_consistency_weighted(pc1, pc2, mask):
    """pc1, pc2 [B, P, n, 3], mask [B, P]: per-part mean squared error, masked mean over parts."""
    d = pc1 - pc2
    per_part = (d * d).sum(-1).mean(-1)
    return (per_part * mask).sum() / mask.sum()
