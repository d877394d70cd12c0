"""Per-launch A/B of two builds of libured_hip.so: every ured_hip.kernels.gemm call of the source
encoder's forward + backward (tools/src_enc_check.py's case) runs on the build in use (URED_LIB),
then again on URED_ALT_LIB into the same (restored) outputs; launches whose outputs differ by
more than --tol (relative to the output's max) are printed with their parameters.

  URED_LIB=build_ab/x.so URED_ALT_LIB=build_ab/y.so python tools/ab_calls.py [--n 128]
"""
import argparse
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import __graft_entry__ as ge  # noqa: E402

ge.add_pkg_path()
from ured_hip import _lib  # noqa: E402
from ured_hip import kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=128)
    ap.add_argument("--tol", type=float, default=1e-4)
    a = ap.parse_args()
    main_h = _lib.lib()
    alt = ctypes.CDLL(os.environ["URED_ALT_LIB"])
    for name, argtypes in _lib._SIGNATURES.items():
        fn = getattr(alt, name)
        fn.argtypes = argtypes
        fn.restype = _lib._RESTYPES.get(name, ctypes.c_int)
    real = K.gemm
    count = [0]

    def wrapped(M, N, Kd, A, lda, B, ldb, C, ldc, **kw):
        outs = {"C": C}
        for k in ("stat_ws", "pool_ws", "bwd_ws"):
            if kw.get(k) is not None:
                outs[k] = kw[k]
        before = {k: v.clone() for k, v in outs.items()}
        real(M, N, Kd, A, lda, B, ldb, C, ldc, **kw)
        mine = {k: v.clone() for k, v in outs.items()}
        for k, v in outs.items():
            v.copy_(before[k])
        _lib._lib = alt
        try:
            real(M, N, Kd, A, lda, B, ldb, C, ldc, **kw)
        finally:
            _lib._lib = main_h
        other = {k: v.clone() for k, v in outs.items()}
        for k, v in outs.items():
            v.copy_(mine[k])
        count[0] += 1
        for k in outs:
            x, y = mine[k], other[k]
            if k == "pool_ws":      # {max, argmax, min, argmin} planes: compare the index planes as ints
                nb = x.shape[0]
                xi, yi = x.view(nb, 4, -1)[:, 1::2].contiguous().view(torch.int32), y.view(nb, 4, -1)[:, 1::2].contiguous().view(torch.int32)
                bad = int((xi != yi).sum())
                if bad:
                    print(f"call {count[0]}: {k} argmax/argmin differ in {bad} entries")
                x, y = x.view(nb, 4, -1)[:, 0::2], y.view(nb, 4, -1)[:, 0::2]
            s = max(float(y.abs().max()), 1e-30)
            e = float((x - y).abs().max()) / s
            if e > a.tol:
                desc = {k2: (tuple(v.shape) if torch.is_tensor(v) else v) for k2, v in kw.items()
                        if v is not None and k2 not in ("bn",)}
                print(f"call {count[0]}: M={M} N={N} K={Kd} lda={lda} ldb={ldb} ldc={ldc} out {k}: rel {e:.3e} "
                      f"{desc}", flush=True)
    K.gemm = wrapped
    import ured_hip.mlp as umlp
    umlp.K.gemm = wrapped
    sys.argv = [sys.argv[0], "--n", str(a.n)]
    import src_enc_check
    src_enc_check.main()
    print(f"{count[0]} gemm calls compared")


if __name__ == "__main__":
    main()
