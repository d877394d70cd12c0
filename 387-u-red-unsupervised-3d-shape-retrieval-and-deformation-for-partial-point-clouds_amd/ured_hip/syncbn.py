"""Optional SyncBN for the data-parallel step (cfg["sync_bn"], default off).

The reference trains on one GPU (README.md:25), so every BatchNorm1d there normalises with the
statistics of the whole batch. Under data parallelism each rank sees 1/world of it; by default
(as DDP does) each rank uses its own batch statistics. With SyncBN every BatchNorm of the
trained nets — the encoders' and residual / reconstruction nets' per-point BNs (ured_hip/mlp.py,
finalized by kernels.bn_fwd_finalize / bn_bwd_finalize) and DeformNet's node BNs
(ured_hip/node.py bn_fwd / bn_bwd) — uses the statistics of the GLOBAL batch, with torch's
SyncBatchNorm semantics (torch/nn/modules/_functions.py):
  forward : each rank's fp64 per-column (count, mean, M2) is all-gathered and merged in rank
            order (Chan), identically on every rank; mean / invstd / the running statistics
            (unbiased with the global count) follow from the merged values;
  backward: the fp64 sums (sum g, sum g*xhat, count) are all-reduced; the input gradient uses
            the global sums, dgamma / dbeta are the rank's local sums (the gradient all-reduce
            of the DP step then averages them, as DDP does with SyncBatchNorm).
Collectives are issued in the same order on every rank (the forward / backward layer order),
through ured_hip/collective.run (so a captured step replays them between graph segments).
The state is process-wide: TrainStep enables it for its process group when cfg["sync_bn"] and
world > 1 (engine/train.py), and a layer in eval mode never synchronises.
"""
import ctypes

import torch
import torch.distributed as dist

from . import _lib, collective

_P, _I, _F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
_lib.register({
    "ured_bn_stats": [_P, _I, _I, _P, _I, _P, _P],
    "ured_bn_finalize_stats": [_P, _I, _P, _P, _F, _F, _P, _P, _P, _P, _P, _P, _P, _P],
    "ured_bn_bwd_sums": [_P, _I, _I, _P, _I, _P, _P],
    "ured_bn_bwd_finalize_sums": [_P, _P, _I, _P, _P, _P, _P, _I, _P, _P, _P, _P],
})

_state = {"group": None, "world": 1}


def enable(group=None):
    """Synchronise BatchNorm statistics over `group` (None: the default process group)."""
    if not dist.is_initialized():
        raise RuntimeError("SyncBN needs an initialised process group")
    _state["group"] = group
    _state["world"] = dist.get_world_size(group)


def disable():
    _state["group"], _state["world"] = None, 1


def active():
    return _state["world"] > 1


def merge_stats(local):
    """local fp64 [..., 3, N] (count, mean, M2) -> the global batch's [..., 3, N]: all-gathered,
    merged in rank order (the same arithmetic on every rank)."""
    local = local.contiguous()
    parts = [torch.empty_like(local) for _ in range(_state["world"])]
    group = _state["group"]
    collective.run(lambda: dist.all_gather(parts, local, group=group))
    st = torch.stack(parts)                               # [world, ..., 3, N]
    c, mu, m2 = st.select(-2, 0), st.select(-2, 1), st.select(-2, 2)
    C = c.sum(0)
    mean = (c * mu).sum(0) / C.clamp(min=1.0)
    M2 = (m2 + c * (mu - mean) ** 2).sum(0)
    return torch.stack([C, mean, M2], dim=-2).contiguous()


def sum_over_ranks(local):
    """local fp64 sums -> their sum over the ranks (a new tensor; `local` is kept)."""
    g = local.clone()
    group = _state["group"]
    collective.run(lambda: dist.all_reduce(g, op=dist.ReduceOp.SUM, group=group))
    return g


def _p(t):
    return None if t is None else t.data_ptr()


def fwd_finalize(stat_ws, M, N, gamma, beta, eps, momentum, running_mean, running_var, rw, nbt, out):
    """The SyncBN form of kernels.bn_fwd_finalize: out = (mean, invstd, scale, shift) [N]."""
    dev = stat_ws.device
    stream = _lib.stream_of(stat_ws)
    local = torch.empty(3, N, dtype=torch.float64, device=dev)
    gw, grows = (None, 0) if rw is None else (rw.w.data_ptr(), rw.group_rows)
    _lib.call("ured_bn_stats", _p(stat_ws), int(M), int(N), gw, grows, _p(local), stream)
    glob = merge_stats(local)
    mean, invstd, scale, shift = out
    _lib.call("ured_bn_finalize_stats", _p(glob), int(N), _p(gamma), _p(beta), float(eps), float(momentum),
              _p(running_mean), _p(running_var), _p(mean), _p(invstd), _p(scale), _p(shift), _p(nbt), stream)


def bwd_finalize(bwd_ws, M, N, gamma, invstd, dgamma, dbeta, rw, coefs):
    """The SyncBN form of kernels.bn_bwd_finalize (coefs = (ca, cb, cc) written)."""
    dev = bwd_ws.device
    stream = _lib.stream_of(bwd_ws)
    local = torch.empty(3, N, dtype=torch.float64, device=dev)
    gw, grows = (None, 0) if rw is None else (rw.w.data_ptr(), rw.group_rows)
    _lib.call("ured_bn_bwd_sums", _p(bwd_ws), int(M), int(N), gw, grows, _p(local), stream)
    glob = sum_over_ranks(local)
    ca, cb, cc = coefs
    _lib.call("ured_bn_bwd_finalize_sums", _p(local), _p(glob), int(N), _p(gamma), _p(invstd), _p(dgamma),
              _p(dbeta), 0, _p(ca), _p(cb), _p(cc), stream)
