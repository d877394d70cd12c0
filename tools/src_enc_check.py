"""Source-encoder forward/backward gradient errors against a float64 oracle run, for the HIP
build in use (URED_LIB) and for the oracle's own fp32 run (tests/test_mlp_gpu.py's case).

  python tools/src_enc_check.py [--n 128]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import __graft_entry__ as ge  # noqa: E402

ge.add_pkg_path()
from oracle import ured_ref  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=128)
    a = ap.parse_args()
    from test_mlp_gpu import _mods, _req
    dev = torch.device("cuda:0")
    P, _, src, _ = _mods(dev)
    Ps = P["src_encoder_all"]
    n = a.n
    g = torch.Generator().manual_seed(n + 1)
    x = torch.rand(2, 3, n, 3, generator=g) - 0.5
    sem = torch.randn(2, 3, 16, generator=g)
    w1, w2 = torch.randn(6, 64, generator=g), torch.randn(6, 64, n, generator=g)
    code, pp = src(x.to(dev), sem.to(dev))
    ((code * w1.to(dev)).sum() + (pp * w2.to(dev)).sum()).backward()
    runs = {}
    for name, dt in (("fp32", torch.float32), ("f64", torch.float64)):
        Q = {k: (v.detach().to(dt) if v.dtype.is_floating_point else v) for k, v in Ps.items()}
        _req(Q)
        rc, rpp = ured_ref.target_encoder(Q, x.to(dt), sem.to(dt), True)
        ((rc * w1.to(dt)).sum() + (rpp * w2.to(dt)).sum()).backward()
        runs[name] = Q
    sd = dict(src.named_parameters())
    print(f"{'param':28s} {'gpu vs f64':>12s} {'cpu32 vs f64':>12s}   (max |d| / max |g64|)")
    for k, v in runs["f64"].items():
        if k.startswith("stn") or not v.dtype.is_floating_point or "running" in k or v.grad is None:
            continue
        r = v.grad
        s = max(r.abs().max().item(), 1e-30)
        eg = (sd[k].grad.detach().double().cpu() - r).abs().max().item() / s
        ec = (runs["fp32"][k].grad.double() - r).abs().max().item() / s
        print(f"{k:28s} {eg:12.3e} {ec:12.3e}")


if __name__ == "__main__":
    main()
