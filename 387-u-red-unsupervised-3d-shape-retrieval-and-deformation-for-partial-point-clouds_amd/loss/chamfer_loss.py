"""Drop-in for the reference loss/chamfer_loss.py (chamfer_distance2, compute_cm_loss).

The reference calls the un-vendored Shape_Measure.distance.ChamferLoss once per
sample and once per part inside Python loops, with a .item() host sync
(loss/chamfer_loss.py:5-30). Here every family of calls is ONE ragged HIP
launch (ured_nn_seg_fwd) with segment tables built on the device:
  full family : out[b, :k_b*1024]  <->  x[b]
  part family : out[b, i*1024:(i+1)*1024]  <->  points of part i of x[b]
ChamferLoss semantics (Shape_Measure is absent, version unpinned): cost1/cost2
are the squared nearest-neighbour distances, as chamfer_3DDist returns them.
"""
import torch

from ured_hip.nn import nn_dense, nn_segments
from ured_hip.ops import PartBatch, build_parts, segment_sum

NP_PER_PART = 1024


class ChamferLoss(torch.nn.Module):
    """Shape_Measure.distance.ChamferLoss stand-in: (p1 [B,n,3], p2 [B,m,3]) -> (cost1 [B,n], cost2 [B,m])."""

    def forward(self, p1, p2):
        d1, d2, _, _ = nn_dense(p1, p2)
        return d1, d2


def chamfer_distance2(p1, p2):
    cost1, cost2 = ChamferLoss()(p1, p2)
    return cost1.mean(dim=1) + cost2.mean(dim=1)


def _as_partbatch(target_p, target_part, mask):
    """Accept our PartBatch or the reference's list (per sample) of lists (per part) of [n_i,3] tensors."""
    if isinstance(target_part, PartBatch):
        return target_part
    B, N, _ = target_p.shape
    P = mask.shape[1]
    xs, labels = [], []
    for b in range(B):
        parts = list(target_part[b])
        xs.append(torch.cat(parts, 0))
        labels.append(torch.cat([torch.full((p.shape[0],), i, device=target_p.device, dtype=torch.long)
                                 for i, p in enumerate(parts)]))
    return build_parts(torch.stack(labels), torch.stack(xs), P)


def _full_segments(B, S, N, k, dev, np_per_part):
    ar = torch.arange(B, device=dev)
    return torch.stack([ar * S, k * np_per_part, ar * N, torch.full_like(ar, N)], 1).int()


def _doubled(parts, B, N, P):
    """The PartBatch of cat([x, x]) (a second copy of the batch: disjoint point ranges)."""
    off = parts.off.long()
    return PartBatch(x_sorted=torch.cat([parts.x_sorted, parts.x_sorted]),
                     off=torch.cat([off[:-1], off[:-1] + B * N, off[-1:] + B * N]).int(),
                     gid=torch.cat([parts.gid, parts.gid + B * P]),
                     counts=torch.cat([parts.counts, parts.counts]), max_parts=P)


def compute_cm_loss_pair(source_p, source_p2, target_p, target_part, mask, np_per_part=NP_PER_PART,
                         return_idx=False):
    """(compute_cm_loss(source_p, ...), compute_cm_loss(source_p2, ...)) against the same
    target — the chamfer and symmetric-chamfer terms of the step (engine/train.py:288,302) — as
    ONE ragged launch per family over the two stacked batches. The NN results are per segment,
    so identical to the separate calls; the row means may round differently by an ulp."""
    B, S, _ = source_p.shape
    N = target_p.shape[1]
    P = mask.shape[1]
    parts = _as_partbatch(target_p, target_part, mask)
    r = compute_cm_loss(torch.cat([source_p, source_p2]), torch.cat([target_p, target_p]),
                        _doubled(parts, B, N, P), torch.cat([mask, mask]), batch_reduction=None,
                        np_per_part=np_per_part, return_idx=return_idx)
    full, part = r[0], r[1]
    # per-half means as one op each, split by unbind (its backward is one stack; slicing the
    # halves would cost a zero-fill + copy per slice and an add)
    f0, f1 = full.view(2, B).mean(1).unbind(0)
    p0, p1 = part.view(2, B).mean(1).unbind(0)
    res = (f0, p0), (f1, p1)
    return res + (r[2][:B],) if return_idx else res


def compute_cm_loss(source_p, target_p, target_part=None, mask=None, batch_reduction="mean",
                    np_per_part=NP_PER_PART, return_idx=False):
    """Returns (mean_b full CD, mean_b part CD) with a mask, else chamfer_distance2 per sample.

    Like the reference, target_part is used only with a mask; CD = mean(cost1) + mean(cost2).
    """
    if mask is None:
        return chamfer_distance2(source_p, target_p)
    B, S, _ = source_p.shape
    N = target_p.shape[1]
    P = mask.shape[1]
    dev = source_p.device
    parts = _as_partbatch(target_p, target_part, mask)
    k = mask.sum(1).round().long()
    src = source_p.contiguous()
    # full family
    segs = _full_segments(B, S, N, k, dev, np_per_part)
    da, _, db, ib = nn_segments(src, target_p.contiguous(), segs, S, N, 3)
    n_valid = (k * np_per_part).clamp(min=1).float()
    full = da.view(B, S).sum(1) / n_valid + db.view(B, N).mean(1)
    full = full.masked_fill(k == 0, float("nan"))
    # part family: part slot i of sample b <-> points of its i-th part (sorted by label)
    slot = torch.arange(P, device=dev)
    valid = slot.unsqueeze(0) < k.unsqueeze(1)
    a_off = (torch.arange(B, device=dev) * S).unsqueeze(1) + slot.unsqueeze(0) * np_per_part
    a_len = valid.long() * np_per_part
    b_off = parts.off[:-1].view(B, P).long()
    b_len = parts.counts * valid
    psegs = torch.stack([a_off, a_len, b_off, b_len], -1).view(B * P, 4).int()
    pa, _, pb, _ = nn_segments(src, parts.x_sorted.contiguous(), psegs, np_per_part, N, 3)
    nchunk = min(S, P * np_per_part) // np_per_part
    pa2 = pa.view(B, S)
    if nchunk * np_per_part != S:      # (a full-width slice would still cost a zero-fill + copy backward)
        pa2 = pa2[:, :nchunk * np_per_part]
    cost1 = pa2.reshape(B, nchunk, np_per_part).mean(-1)
    if nchunk < P:
        cost1 = torch.cat([cost1, cost1.new_zeros(B, P - nchunk)], 1)
    cost2 = segment_sum(pb.view(-1, 1), parts.off, parts.gid).view(B, P) / parts.counts.clamp(min=1).float()
    part_cd = (cost1 + cost2) * valid.float()
    part = part_cd.sum(1) / k.float()
    # return_idx: also the x -> source NN index of every target point ([B, N] int32, relative to
    # the sample's source row) — residual_retrieval_loss's knn_points query, already computed here
    extra = (ib.view(B, N),) if return_idx else ()
    if batch_reduction == "mean":
        return (full.mean(), part.mean()) + extra
    return (full, part) + extra
