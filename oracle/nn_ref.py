"""ctypes wrapper of oracle/nn_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker).

Restates Density_aware_Chamfer_Distance/utils_v2/metrics/CD/chamfer3D/chamfer3D.cu:12-195
on the CPU (see nn_oracle.c for the exact contract). numpy in, numpy out.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libnn_oracle.so")
_lib = None

_F = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_Iptr = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            import subprocess
            os.makedirs(os.path.dirname(LIB_PATH), exist_ok=True)
            subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-fPIC", "-shared",
                                   os.path.join(_HERE, "nn_oracle.c"), "-o", LIB_PATH, "-lm"])
        l = ctypes.CDLL(LIB_PATH)
        c_int = ctypes.c_int
        l.oracle_nn_dir.argtypes = [_F, c_int, _F, c_int, _F, _Iptr]
        l.oracle_nn_fwd.argtypes = [_F, _F, c_int, c_int, c_int, _F, _Iptr, _F, _Iptr]
        l.oracle_nn_bwd.argtypes = [_F, _F, c_int, c_int, c_int, ctypes.c_void_p, ctypes.c_void_p,
                                    _Iptr, _Iptr, _F, _F]
        l.oracle_nn_seg_fwd.argtypes = [_F, _F, _Iptr, c_int, c_int, _F, _Iptr, _F, _Iptr]
        l.oracle_nn_seg_bwd.argtypes = [_F, _F, _Iptr, c_int, ctypes.c_void_p, ctypes.c_void_p,
                                        _Iptr, _Iptr, _F, _F]
        _lib = l
    return _lib


def _f32(x):
    return np.ascontiguousarray(x, dtype=np.float32)


def _i32(x):
    return np.ascontiguousarray(x, dtype=np.int32)


def _vp(x):
    return None if x is None else x.ctypes.data_as(ctypes.c_void_p)


def nn_dir(q, r):
    """queries q [nq,3], refs r [nr,3] -> dist [nq] f32, idx [nq] i32."""
    q, r = _f32(q), _f32(r)
    d = np.zeros(q.shape[0], np.float32)
    i = np.zeros(q.shape[0], np.int32)
    _load().oracle_nn_dir(q, q.shape[0], r, r.shape[0], d, i)
    return d, i


def nn_fwd(xyz1, xyz2):
    """[b,n,3], [b,m,3] -> dist1 [b,n], dist2 [b,m], idx1, idx2 (reference chamfer_3DDist)."""
    xyz1, xyz2 = _f32(xyz1), _f32(xyz2)
    b, n, _ = xyz1.shape
    m = xyz2.shape[1]
    d1 = np.zeros((b, n), np.float32); d2 = np.zeros((b, m), np.float32)
    i1 = np.zeros((b, n), np.int32); i2 = np.zeros((b, m), np.int32)
    _load().oracle_nn_fwd(xyz1, xyz2, b, n, m, d1, i1, d2, i2)
    return d1, d2, i1, i2


def nn_bwd(xyz1, xyz2, gd1, gd2, idx1, idx2):
    xyz1, xyz2 = _f32(xyz1), _f32(xyz2)
    b, n, _ = xyz1.shape
    m = xyz2.shape[1]
    gd1 = None if gd1 is None else _f32(gd1)
    gd2 = None if gd2 is None else _f32(gd2)
    g1 = np.zeros_like(xyz1); g2 = np.zeros_like(xyz2)
    _load().oracle_nn_bwd(xyz1, xyz2, b, n, m, _vp(gd1), _vp(gd2), _i32(idx1), _i32(idx2), g1, g2)
    return g1, g2


def nn_seg_fwd(a, b, segs, dirs=3):
    a, b, segs = _f32(a).reshape(-1, 3), _f32(b).reshape(-1, 3), _i32(segs).reshape(-1, 4)
    da = np.zeros(a.shape[0], np.float32); ia = np.zeros(a.shape[0], np.int32)
    db = np.zeros(b.shape[0], np.float32); ib = np.zeros(b.shape[0], np.int32)
    _load().oracle_nn_seg_fwd(a, b, segs, segs.shape[0], dirs, da, ia, db, ib)
    return da, ia, db, ib


def nn_seg_bwd(a, b, segs, gd_a, gd_b, idx_a, idx_b):
    a, b, segs = _f32(a).reshape(-1, 3), _f32(b).reshape(-1, 3), _i32(segs).reshape(-1, 4)
    gd_a = None if gd_a is None else _f32(gd_a)
    gd_b = None if gd_b is None else _f32(gd_b)
    ga = np.zeros_like(a); gb = np.zeros_like(b)
    _load().oracle_nn_seg_bwd(a, b, segs, segs.shape[0], _vp(gd_a), _vp(gd_b), _i32(idx_a), _i32(idx_b), ga, gb)
    return ga, gb


def dist_chamfer(a, b):
    """Restatement of the reference's Python chamfer, Density_aware_Chamfer_Distance/utils_v2/
    metrics/CD/chamfer_python.py:18-39 (distChamfer): the dense float64 B x n x m matrix by the
    expansion |x|^2 + |y|^2 - 2 x.y, min / argmin along both axes, cast to float32 / int32.
    a [B,n,d], b [B,m,d] torch tensors. Used as the CPU baseline's chamfer (bench.py)."""
    import torch
    x, y = a.double(), b.double()
    xx = (x * x).sum(2)
    yy = (y * y).sum(2)
    zz = torch.bmm(x, y.transpose(2, 1))
    P = xx.unsqueeze(2) + yy.unsqueeze(1) - 2 * zz
    m1, i1 = torch.min(P, 2)
    m2, i2 = torch.min(P, 1)
    return m1.float(), m2.float(), i1.int(), i2.int()
