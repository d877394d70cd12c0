"""Drop-in for the reference loss/basic_loss.py: residual_retrieval_loss (basic_loss.py:249-265)
and a pytorch3d.ops.knn_points(K=1) subset.

pytorch3d is absent from the reference tree (version unpinned); the K=1 query
here is the x -> source direction of the same HIP nearest-neighbour primitive
(squared L2, lowest index on ties), one ragged launch for the whole batch.
"""
from collections import namedtuple

import torch

from ured_hip.nn import nn_segments

NP_PER_PART = 1024
KNN = namedtuple("KNN", ["dists", "idx", "knn"])


def knn_points(p1, p2, lengths1=None, lengths2=None, K=1, return_nn=False, **_):
    """K=1 nearest neighbour of every p1 point among p2 (pytorch3d.ops.knn_points subset).

    p1 [B,n,3], p2 [B,m,3]; lengths2 [B] limits the valid p2 points per sample.
    Returns dists [B,n,1] (squared), idx [B,n,1] (int64), knn [B,n,1,3] if return_nn.
    """
    if K != 1:
        raise NotImplementedError("only K=1 is on the U-RED path (loss/basic_loss.py:257)")
    B, n, _ = p1.shape
    m = p2.shape[1]
    dev = p1.device
    ar = torch.arange(B, device=dev)
    n1 = torch.full_like(ar, n) if lengths1 is None else lengths1.to(dev).long()
    n2 = torch.full_like(ar, m) if lengths2 is None else lengths2.to(dev).long()
    segs = torch.stack([ar * m, n2, ar * n, n1], 1).int()
    _, _, d, i = nn_segments(p2.contiguous(), p1.contiguous(), segs, m, n, 2)
    d, i = d.view(B, n, 1), i.view(B, n, 1).long()
    nn = torch.gather(p2, 1, i.expand(-1, -1, 3)).unsqueeze(2) if return_nn else None
    return KNN(d, i, nn)


def residual_retrieval_loss(x, x_source, residuals, mask_part=None, np_per_part=NP_PER_PART, nn_idx=None):
    """x [B,N,3] target, x_source [B,S,3] deformed sources (only the first k_b*1024 are valid),
    residuals [B,N,3] -> (mean_n sum_xyz |x + r - nn|, mean_n sum_xyz |r|).
    nn_idx [B,N] (optional): the x -> x_source nearest-neighbour indices when the caller already
    has them (the chamfer full family computes exactly this query, compute_cm_loss(return_idx))."""
    B, S, _ = x_source.shape
    if nn_idx is None:
        valid = (mask_part.sum(1).round().long() * np_per_part).clamp(max=S)
        _, _, nn = knn_points(x, x_source, lengths2=valid, K=1, return_nn=True)
        nn = nn.squeeze(2)
    else:
        nn = torch.gather(x_source, 1, nn_idx.long().unsqueeze(-1).expand(-1, -1, 3))
    res_nn = x + residuals - nn
    return torch.abs(res_nn).sum(-1).mean(), torch.abs(residuals).sum(-1).mean()
