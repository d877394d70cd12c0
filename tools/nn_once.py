"""Two-pass NN forward, both directions, on one dense shape, 20 graph-replayed calls (for counter passes).

  python tools/nn_once.py [B n m]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402


def main():
    from ured_hip import nn as unn
    unn.FUSED = False
    B, n, m = (int(v) for v in sys.argv[1:4]) if len(sys.argv) >= 4 else (16, 2048, 2048)
    r = bench.chamfer_rate(torch.device("cuda:0"), B, n, m, iters=20)
    print(r["shape"], r["ms"], flush=True)


if __name__ == "__main__":
    main()
