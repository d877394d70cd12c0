"""NN forward on the train step's ragged families and the micro-benchmark shapes, for A/B of
fused-plan variants (run once per library build via URED_LIB).

  URED_LIB=build_ab/lib_x.so python tools/nn_seg_ab.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402
ge.add_pkg_path()
import torch  # noqa: E402
from ured_hip import nn as unn  # noqa: E402


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    B, S, N, k = 16, 16384, 2048, 4
    out = torch.rand(B, S, 3, generator=g).to(dev)
    x = torch.rand(B, N, 3, generator=g).to(dev)
    ar = torch.arange(B)
    full = torch.stack([ar * S, torch.full((B,), k * 1024), ar * N, torch.full((B,), N)], 1).int().to(dev)
    P = 16
    slot = torch.arange(P)
    a_off = (ar * S).unsqueeze(1) + slot.unsqueeze(0) * 1024
    valid = slot.unsqueeze(0) < k
    a_len = torch.where(valid, torch.full_like(a_off, 1024), torch.zeros_like(a_off))
    b_len = torch.where(valid, torch.full_like(a_off, N // k), torch.zeros_like(a_off))
    b_off = (ar * N).unsqueeze(1) + slot.unsqueeze(0) * (N // k)
    part = torch.stack([a_off, a_len, b_off, b_len], -1).view(B * P, 4).int().to(dev)
    res = {"lib": os.environ.get("URED_LIB", "default")}
    res["full_us"] = round(timeit(lambda: unn.nn_segments(out, x, full, S, N, 3)), 2)
    res["part_us"] = round(timeit(lambda: unn.nn_segments(out, x, part, 1024, N, 3)), 2)
    for (b, n, m) in [(16, 2048, 2048), (64, 4096, 4096), (16, 16384, 2048), (4096, 1024, 1024)]:
        p1 = torch.rand(b, n, 3, generator=g).to(dev)
        p2 = torch.rand(b, m, 3, generator=g).to(dev)
        t = timeit(lambda: unn.nn_dense(p1, p2), 10)
        res[f"{b}x{n}x{m}_gpair_s"] = round(b * n * m / (t * 1e-6) / 1e9, 1)
    unn.FUSED = False
    res["full_two_pass_us"] = round(timeit(lambda: unn.nn_segments(out, x, full, S, N, 3)), 2)
    res["part_two_pass_us"] = round(timeit(lambda: unn.nn_segments(out, x, part, 1024, N, 3)), 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
