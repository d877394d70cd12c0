"""Drop-in for Density_aware_Chamfer_Distance/utils_v2/metrics/EMD/emd_module.py (emdFunction,
emdModule): the auction EMD on libured_hip.so (csrc/emd.hip) instead of the JIT-built CUDA
extension. Same inputs / outputs: xyz1, xyz2 [b, n, 3] (equal sizes), eps, iters ->
dist [b, n] (squared distance to the matched point), assignment [b, n] int32; gradient for
xyz1 only. Deterministic (see csrc/emd.hip); n need not be a multiple of 1024 here.
"""
import torch
from torch import nn
from torch.autograd import Function

from ured_hip import _lib


class emdFunction(Function):
    @staticmethod
    def forward(ctx, xyz1, xyz2, eps, iters):
        b, n, _ = xyz1.size()
        _, m, _ = xyz2.size()
        if n != m or xyz1.size(0) != xyz2.size(0):
            raise ValueError(f"emd: the two clouds must have the same shape, got {tuple(xyz1.shape)} {tuple(xyz2.shape)}")
        _lib.require_device(xyz1, xyz2)
        xyz1 = xyz1.contiguous().float()
        xyz2 = xyz2.contiguous().float()
        dist = torch.empty(b, n, device=xyz1.device)
        assignment = torch.empty(b, n, device=xyz1.device, dtype=torch.int32)
        nbytes = _lib.query("ured_emd_workspace", b, n)
        ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=xyz1.device)
        _lib.call("ured_emd_fwd", _lib.ptr(xyz1), _lib.ptr(xyz2), b, n, float(eps), int(iters),
                  _lib.ptr(dist), _lib.ptr(assignment), _lib.ptr(ws), nbytes, _lib.stream_of(xyz1))
        ctx.save_for_backward(xyz1, xyz2, assignment)
        ctx.mark_non_differentiable(assignment)
        return dist, assignment

    @staticmethod
    def backward(ctx, graddist, _gradidx):
        xyz1, xyz2, assignment = ctx.saved_tensors
        b, n, _ = xyz1.shape
        gradxyz1 = torch.zeros_like(xyz1)
        gradxyz2 = torch.zeros_like(xyz2)
        if graddist is not None:
            _lib.call("ured_emd_bwd", _lib.ptr(xyz1), _lib.ptr(xyz2), b, n, _lib.ptr(graddist.contiguous()),
                      _lib.ptr(assignment), _lib.ptr(gradxyz1), _lib.stream_of(xyz1))
        return gradxyz1, gradxyz2, None, None


class emdModule(nn.Module):
    def forward(self, input1, input2, eps, iters):
        return emdFunction.apply(input1, input2, eps, iters)
