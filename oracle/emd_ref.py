"""ctypes wrapper of oracle/emd_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker for the
HIP auction EMD; see emd_oracle.c for the reference lines it restates)."""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libemd_oracle.so")
_F = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_I = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            os.makedirs(os.path.dirname(LIB_PATH), exist_ok=True)
            subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-fPIC", "-shared",
                                   os.path.join(_HERE, "emd_oracle.c"), "-o", LIB_PATH, "-lm"])
        lib = ctypes.CDLL(LIB_PATH)
        lib.oracle_emd_fwd.argtypes = [_F, _F, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_int, _F, _I]
        lib.oracle_emd_fwd.restype = None
        _lib = lib
    return _lib


def emd_fwd(xyz1, xyz2, eps, iters):
    """-> (dist [b,n] float32, assignment [b,n] int32)."""
    x1 = np.ascontiguousarray(xyz1, np.float32)
    x2 = np.ascontiguousarray(xyz2, np.float32)
    b, n, _ = x1.shape
    assert x2.shape == x1.shape
    dist = np.zeros((b, n), np.float32)
    asg = np.zeros((b, n), np.int32)
    _load().oracle_emd_fwd(x1, x2, b, n, float(eps), int(iters), dist, asg)
    return dist, asg
