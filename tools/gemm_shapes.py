"""Print the GEMM launch shapes of one bench step (URED_GEMM_SHAPES=1) with FLOPs, tiles and
the tile-quantisation efficiency (useful MACs / MACs of the padded 128x128 tiles)."""
import os
import sys
from collections import Counter

os.environ["URED_GEMM_SHAPES"] = "1"
sys.argv = [sys.argv[0], "--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--no-breakdown",
            "--no-all-slots-rate", "--no-extras"]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from ured_hip import kernels as K  # noqa: E402

K._SHAPE_LOG.clear()
bench.main()
log = K._SHAPE_LOG[len(K._SHAPE_LOG) // 3:] if False else K._SHAPE_LOG
c = Counter(log)
tot = 0
rows = []
for (M, N, Kd, akm, bkm, pa, pb, epi, sp), n in c.items():
    fl = 2.0 * M * N * Kd * n
    tiles = -(-M // 128) * -(-N // 128)
    eff = M * N / (tiles * 128 * 128)
    rows.append((fl, M, N, Kd, akm, bkm, pa, pb, epi, sp, n, tiles, eff))
    tot += fl
for r in sorted(rows, reverse=True):
    fl, M, N, Kd, akm, bkm, pa, pb, epi, sp, n, tiles, eff = r
    kind = f"<{int(akm)},{int(bkm)},{pa},{pb},{epi}>"
    print(f"{fl / tot * 100:5.1f}%  {kind:14s} M={M:6d} N={N:5d} K={Kd:6d} splits={sp:3d} x{n:3d} tiles={tiles:5d} eff={eff:.3f}")
