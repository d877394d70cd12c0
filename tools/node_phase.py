"""Per-workgroup phase timing of one node-GEMM launch in DeformNet_MatchingNet's forward + backward
(the training step's shape: B = 16, C = 512, 16 part slots).

Needs the timing build, e.g. bash tools/build_ab.sh nts -DURED_NODE_TIMING=1 -DURED_NTS_M=288
-DURED_NTS_N=1536 -DURED_NTS_K=512, then URED_LIB=build_ab/nts.so python tools/node_phase.py.
Reads the last recorded launch whose first job has that shape: per workgroup (wave 0) the real-time
clock (100 MHz) at start, first K-chunk landed, MFMA loop end, partial tiles summed in LDS, stores done.
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

ge.add_pkg_path()


def main():
    from network.deformation_net import DeformNet_MatchingNet
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    C = 512
    net = DeformNet_MatchingNet(3 * C, graph_dim=C, max_num_parts=16, matching=False).to(dev).train()
    tf = torch.randn(16, C, device=dev, requires_grad=True)
    sp = torch.randn(16, 16, C, device=dev, requires_grad=True)
    for _ in range(3):
        out = net(tf, sp, None)
        out.sum().backward()
    torch.cuda.synchronize()
    lib = ctypes.CDLL(os.environ["URED_LIB"])
    n = 4096
    buf = (ctypes.c_ulonglong * (n * 8))()
    assert lib.ured_debug_node_ts(buf, n) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(n, 8)
    a = a[a[:, 7] == 1]
    if len(a) == 0:
        print("no workgroup recorded (shape not launched?)")
        return
    t = a[:, :5].astype(np.int64)
    t = (t - t[:, 0].min()) * 10e-3
    print(f"workgroups {len(a)}  launch span {t[:, 4].max():.2f} us  (first start -> last end)")
    for name, v in (("start skew", t[:, 0]), ("start -> first chunk landed", t[:, 1] - t[:, 0]),
                    ("chunk loop (MFMAs + later chunks)", t[:, 2] - t[:, 1]),
                    ("partials to LDS + barrier", t[:, 3] - t[:, 2]), ("combine + epilogue stores", t[:, 4] - t[:, 3]),
                    ("whole workgroup", t[:, 4] - t[:, 0])):
        print(f"  {name:34s} mean {v.mean():6.2f}  p10 {np.percentile(v, 10):6.2f}  p50 {np.percentile(v, 50):6.2f}  "
              f"p90 {np.percentile(v, 90):6.2f} us")


if __name__ == "__main__":
    main()
