"""Per-kernel cost of short launches replayed from a HIP graph: 200 back-to-back launches of
(a) ured_copy_batch on 4 bytes (one workgroup), (b) a torch fill_ of one element, (c) ured_copy_batch
on 4 MB (2048 workgroups), each captured in a graph and replayed; HIP events around the replays.
Compare with the same launches' durations in a rocprofv3 kernel trace.

  python tools/launch_floor.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

ge.add_pkg_path()


def per_launch_us(fn, n=200, reps=5):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / (reps * n)


def main():
    from ured_hip.ops import copy_batch
    dev = torch.device("cuda:0")
    a, b = torch.zeros(1, device=dev), torch.ones(1, device=dev)
    big_a, big_b = torch.zeros(1 << 20, device=dev), torch.ones(1 << 20, device=dev)
    print(f"copy_batch 4 B     : {per_launch_us(lambda: copy_batch([(a, b)])):6.2f} us/launch", flush=True)
    print(f"torch fill_ 1 elem : {per_launch_us(lambda: a.fill_(2.0)):6.2f} us/launch", flush=True)
    print(f"copy_batch 4 MB    : {per_launch_us(lambda: copy_batch([(big_a, big_b)])):6.2f} us/launch", flush=True)


if __name__ == "__main__":
    main()
