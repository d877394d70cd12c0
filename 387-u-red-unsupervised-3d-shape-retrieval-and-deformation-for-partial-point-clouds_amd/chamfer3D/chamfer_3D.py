"""The `chamfer_3D` extension module itself, on libured_hip.so.

The reference JIT-builds a pybind11 module named `chamfer_3D` from chamfer_cuda.cpp +
chamfer3D.cu (dist_chamfer_3D.py:11-17) whose two functions are called with caller-allocated
tensors (chamfer_cuda.cpp:17-33):

  forward(xyz1 [b,n,3], xyz2 [b,m,3], dist1 [b,n], dist2 [b,m], idx1 [b,n] i32, idx2 [b,m] i32) -> 1
  backward(xyz1, xyz2, gradxyz1, gradxyz2, graddist1, graddist2, idx1, idx2) -> 1

forward overwrites dist/idx; backward ACCUMULATES into gradxyz1/gradxyz2 (the caller zeroes
them, chamfer3D.cu:166-171). Same contract here (float32 contiguous CUDA tensors, int32
indices, squared distances, lowest index on ties), through the C-ABI entry points ured_nn_fwd /
ured_nn_bwd on the current torch stream. Differences: a failed launch raises (the reference
printed and returned 0, chamfer3D.cu:145-151), and the backward is deterministic.
So `import chamfer_3D` resolves to this module for reference code that imports it directly.
"""
import torch

from ured_hip import _lib


def _check(name, t, dtype, shape=None):
    if not torch.is_tensor(t) or t.dtype != dtype or not t.is_contiguous():
        raise TypeError(f"chamfer_3D: {name} must be a contiguous {dtype} tensor")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"chamfer_3D: {name} has shape {tuple(t.shape)}, expected {tuple(shape)}")


def _shapes(xyz1, xyz2):
    if xyz1.dim() != 3 or xyz2.dim() != 3 or xyz1.shape[2] != 3 or xyz2.shape[2] != 3 or xyz1.shape[0] != xyz2.shape[0]:
        raise ValueError(f"chamfer_3D: expected [b,n,3] and [b,m,3], got {tuple(xyz1.shape)} {tuple(xyz2.shape)}")
    return xyz1.shape[0], xyz1.shape[1], xyz2.shape[1]


def forward(xyz1, xyz2, dist1, dist2, idx1, idx2):
    b, n, m = _shapes(xyz1, xyz2)
    for name, t, dt, sh in (("xyz1", xyz1, torch.float32, None), ("xyz2", xyz2, torch.float32, None),
                            ("dist1", dist1, torch.float32, (b, n)), ("dist2", dist2, torch.float32, (b, m)),
                            ("idx1", idx1, torch.int32, (b, n)), ("idx2", idx2, torch.int32, (b, m))):
        _check(name, t, dt, sh)
    _lib.require_device(xyz1, xyz2, dist1, dist2, idx1, idx2)
    if n and m:
        _lib.call("ured_nn_fwd", _lib.ptr(xyz1), _lib.ptr(xyz2), b, n, m, 3, _lib.ptr(dist1), _lib.ptr(idx1),
                  _lib.ptr(dist2), _lib.ptr(idx2), _lib.stream_of(xyz1))
    return 1


def backward(xyz1, xyz2, gradxyz1, gradxyz2, graddist1, graddist2, idx1, idx2):
    b, n, m = _shapes(xyz1, xyz2)
    for name, t, dt, sh in (("xyz1", xyz1, torch.float32, None), ("xyz2", xyz2, torch.float32, None),
                            ("gradxyz1", gradxyz1, torch.float32, (b, n, 3)),
                            ("gradxyz2", gradxyz2, torch.float32, (b, m, 3)),
                            ("graddist1", graddist1, torch.float32, (b, n)),
                            ("graddist2", graddist2, torch.float32, (b, m)),
                            ("idx1", idx1, torch.int32, (b, n)), ("idx2", idx2, torch.int32, (b, m))):
        _check(name, t, dt, sh)
    _lib.require_device(xyz1, xyz2, gradxyz1, gradxyz2, graddist1, graddist2, idx1, idx2)
    if n and m:
        _lib.call("ured_nn_bwd", _lib.ptr(xyz1), _lib.ptr(xyz2), b, n, m, _lib.ptr(graddist1), _lib.ptr(graddist2),
                  _lib.ptr(idx1), _lib.ptr(idx2), _lib.ptr(gradxyz1), _lib.ptr(gradxyz2), _lib.stream_of(xyz1))
    return 1
