"""Which phase of the source-encoder step makes two builds disagree: forward on build X, backward on
build Y (X, Y in {URED_LIB, URED_ALT_LIB}); gradient errors against a float64 oracle run.

  URED_LIB=build_ab/x.so URED_ALT_LIB=build_ab/y.so python tools/ab_phase.py [--n 128]
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
from oracle import ured_ref  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=128)
    a = ap.parse_args()
    from test_mlp_gpu import _mods, _req
    libs = {"main": _lib.lib()}
    alt = ctypes.CDLL(os.environ["URED_ALT_LIB"])
    for name, argtypes in _lib._SIGNATURES.items():
        fn = getattr(alt, name)
        fn.argtypes = argtypes
        fn.restype = _lib._RESTYPES.get(name, ctypes.c_int)
    libs["alt"] = alt
    dev = torch.device("cuda:0")
    n = a.n
    g = torch.Generator().manual_seed(n + 1)
    x = torch.rand(2, 3, n, 3, generator=g) - 0.5
    sem = torch.randn(2, 3, 16, generator=g)
    w1, w2 = torch.randn(6, 64, generator=g), torch.randn(6, 64, n, generator=g)
    P, _, _, _ = _mods(dev)
    Q = {k: (v.detach().double() if v.dtype.is_floating_point else v) for k, v in P["src_encoder_all"].items()}
    _req(Q)
    rc, rpp = ured_ref.target_encoder(Q, x.double(), sem.double(), True)
    ((rc * w1.double()).sum() + (rpp * w2.double()).sum()).backward()
    for fwd, bwd in (("main", "main"), ("alt", "alt"), ("main", "alt"), ("alt", "main")):
        _, _, src, _ = _mods(dev)
        _lib._lib = libs[fwd]
        code, pp = src(x.to(dev), sem.to(dev))
        torch.cuda.synchronize()
        _lib._lib = libs[bwd]
        ((code * w1.to(dev)).sum() + (pp * w2.to(dev)).sum()).backward()
        torch.cuda.synchronize()
        _lib._lib = libs["main"]
        sd = dict(src.named_parameters())
        worst = max((float((sd[k].grad.double().cpu() - v.grad).abs().max()) / max(float(v.grad.abs().max()), 1e-30), k)
                    for k, v in Q.items() if v.grad is not None and k in sd and not k.endswith(".bias"))
        print(f"forward {fwd:4s} backward {bwd:4s}: worst weight-gradient error vs float64 {worst[0]:.3e} ({worst[1]})",
              flush=True)


if __name__ == "__main__" and not os.environ.get("AB_FWD"):
    main()


def forward_diff():
    """Forward intermediates of the two builds side by side (same module weights and inputs)."""
    from test_mlp_gpu import _mods
    alt = ctypes.CDLL(os.environ["URED_ALT_LIB"])
    for name, argtypes in _lib._SIGNATURES.items():
        fn = getattr(alt, name)
        fn.argtypes = argtypes
        fn.restype = _lib._RESTYPES.get(name, ctypes.c_int)
    main_h = _lib.lib()
    dev = torch.device("cuda:0")
    n = 128
    g = torch.Generator().manual_seed(n + 1)
    x = torch.rand(2, 3, n, 3, generator=g) - 0.5
    sem = torch.randn(2, 3, 16, generator=g)
    outs = []
    for h in (main_h, alt):
        _, _, src, _ = _mods(dev)
        _lib._lib = h
        code, pp = src(x.to(dev), sem.to(dev))
        torch.cuda.synchronize()
        fn = code.grad_fn
        sv = fn.saved_tensors
        outs.append((code.detach(), pp.detach(), sv[3].clone(), [t.clone() for t in sv[4:11]],
                     [(s.mean.clone(), s.invstd.clone(), s.scale.clone(), s.shift.clone()) for s in fn.states]))
    _lib._lib = main_h
    (c0, p0, a0, Y0, S0), (c1, p1, a1, Y1, S1) = outs
    r = lambda u, v: float((u - v).abs().max() / max(float(v.abs().max()), 1e-30))
    print(f"code {r(c0, c1):.2e} pp {r(p0, p1):.2e} pool argidx differ {int((a0 != a1).sum())} of {a0.numel()}")
    for i in range(7):
        print(f"layer {i}: Y {r(Y0[i], Y1[i]):.2e}  mean {r(S0[i][0], S1[i][0]):.2e}  invstd {r(S0[i][1], S1[i][1]):.2e}"
              f"  scale {r(S0[i][2], S1[i][2]):.2e}  shift {r(S0[i][3], S1[i][3]):.2e}")
    if int((a0 != a1).sum()):
        idx = (a0 != a1).nonzero()[:5]
        Y5 = Y1[5]
        for gi, ch in idx.tolist():
            r0, r1 = int(a0[gi, ch]), int(a1[gi, ch])
            print(f"  group {gi} ch {ch}: rows {r0} vs {r1}; y5 there {float(Y5[r0, ch]):.9g} {float(Y5[r1, ch]):.9g}"
                  f" scale {float(S1[5][2][ch]):.3g}")


if __name__ == "__main__" and os.environ.get("AB_FWD"):
    forward_diff()
