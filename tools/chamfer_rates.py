"""NN forward (both directions) rates at a few dense shapes, graph-replayed (bench.chamfer_rate),
with the fused path allowed and, for comparison, forced off (two-pass at every size).

  python tools/chamfer_rates.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402

SHAPES = [(16, 2048, 2048), (2, 512, 512), (32, 2000, 1000), (8, 4096, 4096), (16, 4096, 4096), (64, 4096, 4096)]


def main():
    from ured_hip import nn as unn
    dev = torch.device("cuda:0")
    for fused in (True, False):
        unn.FUSED = fused
        for shp in SHAPES:
            r = bench.chamfer_rate(dev, *shp, iters=10)
            path = r["path"] if fused else "two-pass"
            print(json.dumps({"shape": r["shape"], "ms": r["ms"], "gpair_dist_s": r["gpair_dist_s"], "path": path}),
                  flush=True)


if __name__ == "__main__":
    main()
