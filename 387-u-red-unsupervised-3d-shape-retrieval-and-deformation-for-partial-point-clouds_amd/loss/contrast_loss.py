"""Drop-in for the reference loss/contrast_loss.py (InfoNCE between target part features and
source part codes; contrast_loss.py:35-102).

Data-parallel semantics: with a process group the source codes are gathered from
every rank. The reference's dist.all_gather is not autograd-aware (the gathered
copies carry no gradient, contrast_loss.py:35-58); that is the default here too.
differentiable=True keeps this rank's own slice in the graph instead.
"""
import math

import torch
import torch.distributed as dist
import torch.nn.functional as F


def is_dist_avail_and_initialized():
    return dist.is_available() and dist.is_initialized()


def get_world_size():
    return dist.get_world_size() if is_dist_avail_and_initialized() else 1


def get_rank():
    return dist.get_rank() if is_dist_avail_and_initialized() else 0


def gathers(force=False):
    """Whether the source codes go through a collective: world > 1, or `force` (engine/dp.py
    DataParallelStep with cfg["dp_force_collectives"] passes it per step, so a one-GPU box
    exercises the collective path without changing any other step in the process)."""
    return get_world_size() > 1 or (force and is_dist_avail_and_initialized())


def all_gather_batch(tensors, differentiable=False, force=False):
    world = get_world_size()
    if not gathers(force):
        return tensors
    from ured_hip import collective
    out = []
    for t in tensors:
        bufs = [torch.empty_like(t) for _ in range(world)]
        # detached: the closure lives as long as a captured step that replays it, and a tensor
        # with autograd history would keep that step's autograd graph (and the AccumulateGrad
        # nodes, bound to the capture's stream) alive into later captures (engine/dp.py)
        tc = t.detach().contiguous()
        # eager, or between two segments of a captured step (ured_hip/collective.py)
        collective.run(lambda bufs=bufs, tc=tc: dist.all_gather(bufs, tc))
        if differentiable:
            bufs[get_rank()] = t
        out.append(torch.cat(bufs, 0))
    return out


LOGIT_SCALE = math.log(1 / 0.07)
_SCALE32 = float(torch.tensor(LOGIT_SCALE, dtype=torch.float32).exp())


def compute_contrast_loss_loss(tgt_part_f, src_f, src_labels, differentiable_gather=False, force_gather=False):
    bs, num_part = src_f.shape[0], src_f.shape[1]
    t = tgt_part_f.reshape(bs * num_part, -1)
    s = src_f.reshape(bs * num_part, -1)
    n = bs * num_part
    labels = (n * get_rank() + torch.arange(n, device=t.device)).masked_fill_(src_labels.reshape(n).to(t.device) == -1, -1)
    t_e = F.normalize(t, dim=-1, p=2)
    s_e = F.normalize(s, dim=-1, p=2)
    # the reference gathers [t_e, s_e] and discards the gathered t_e (contrast_loss.py:35-58):
    # only the source codes are gathered here (same logits, one collective fewer)
    (s_all,) = all_gather_batch([s_e], differentiable=differentiable_gather, force=force_gather)
    scale = _SCALE32                    # exp(logit scale) rounded to fp32 once, as the fp32 tensor exp would
    if t_e.is_cuda:
        # logits t_e s_all^T on the node GEMM (csrc/node.hip): forward and both backward GEMMs
        from ured_hip.node import node_linear
        return F.cross_entropy(node_linear(scale * t_e, s_all), labels, ignore_index=-1)
    return F.cross_entropy(scale * t_e @ s_all.t(), labels, ignore_index=-1)
