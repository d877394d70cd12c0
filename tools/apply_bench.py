"""BN-backward apply (bn_bwd_apply4_kernel) against the plain read-two-write-one rate of the same
tensors: torch.add(G, Y, out=dY) (PyTorch's vectorized elementwise kernel) and a float4 copy.
If the apply runs at the add's rate, the pass sits at the memory system's ceiling for its bytes.

  python tools/apply_bench.py [--iters 30]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

ge.add_pkg_path()
from ured_hip import _lib  # noqa: E402
from ured_hip import kernels as K  # noqa: E402

SHAPES = [(62464, 1024), (62464, 512), (32768, 1024), (32768, 512), (32768, 256), (62464, 128)]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    ge.build()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    out = {}
    for M, N in SHAPES:
        G = torch.randn(M, N, device=dev, generator=g)
        Y = torch.randn(M, N, device=dev, generator=g)
        dY = torch.empty_like(Y)
        cs = torch.empty(K.nblocks(M), N, device=dev)
        mean = torch.randn(N, device=dev, generator=g) * 0.1
        ca, cb, cc = (torch.randn(N, device=dev, generator=g) for _ in range(3))
        st = _lib.stream_of(Y)

        def apply(res=0, colsum=True):
            _lib.call("ured_bn_bwd_apply", K._p(G), K._p(Y), M, N, N, res, K._p(mean), K._p(ca), K._p(cb),
                      K._p(cc), K._p(dY), K._p(cs) if colsum else None, None, 0, st)

        byts = 3.0 * M * N * 4
        r = {"apply": byts / timeit(apply, a.iters) / 1e9,
             "apply_res": byts / timeit(lambda: apply(1), a.iters) / 1e9,
             "apply_no_colsum": byts / timeit(lambda: apply(0, False), a.iters) / 1e9,
             "torch_add": byts / timeit(lambda: torch.add(G, Y, out=dY), a.iters) / 1e9,
             "torch_copy(2x traffic/3)": 2.0 * M * N * 4 / timeit(lambda: dY.copy_(G), a.iters) / 1e9}
        name = f"{M}x{N}"
        out[name] = {k: round(v, 0) for k, v in r.items()}
        print(name, "GB/s (algorithmic bytes)", out[name], flush=True)
        del G, Y, dY, cs
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
