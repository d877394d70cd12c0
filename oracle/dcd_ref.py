"""CPU restatement of the density-aware chamfer and the offline all-pairs pseudo-label
generation. TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench cpu_baseline):
never imported by the product package.

  calc_cd   <- Density_aware_Chamfer_Distance/utils_v2/model_utils.py:53-70
  calc_dcd  <- Density_aware_Chamfer_Distance/utils_v2/model_utils.py:13-51
  pair rows <- engine/generate_pair.py:69-85 (get_src_pair: row i vs clouds j >= i,
               compute_dcd_loss(dataset[j], dataset[i]) = calc_dcd(x=cloud j, gt=cloud i),
               engine/geometry_utils.py:80-82)
  connect   <- engine/visualization.py:30-46 (upper-triangular rows, M + M.T; the
               diagonal is counted twice, as in the reference)

The NN is the C oracle (nn_ref, the fp32 direct-difference formula of chamfer3D.cu).
Arithmetic is float32 elementwise like the reference's torch ops; the means use numpy's
pairwise float32 sum, so parity with the GPU kernel (fixed tree order) is to ~1e-6.
Pinned against tests/golden/dcd.npz (the reference's calc_dcd run on the reference's
own float64 distChamfer).
"""
import numpy as np

from . import nn_ref


def calc_cd(output, gt):
    """model_utils.py:53-60: cham_loss(gt, output) -> dist1 is gt -> output."""
    d1, d2, i1, i2 = nn_ref.nn_fwd(gt, output)
    cd_p = (np.sqrt(d1).mean(1, dtype=np.float32) + np.sqrt(d2).mean(1, dtype=np.float32)) / np.float32(2)
    cd_t = d1.mean(1, dtype=np.float32) + d2.mean(1, dtype=np.float32)
    return cd_p, cd_t, d1, d2, i1, i2


def calc_dcd(x, gt, alpha=1000, n_lambda=1, non_reg=False):
    x = np.asarray(x, np.float32)
    gt = np.asarray(gt, np.float32)
    n_x, n_gt = x.shape[1], gt.shape[1]
    if non_reg:
        frac_12, frac_21 = max(1, n_x / n_gt), max(1, n_gt / n_x)
    else:
        frac_12, frac_21 = n_x / n_gt, n_gt / n_x
    cd_p, cd_t, d1, d2, i1, i2 = calc_cd(x, gt)
    f32 = np.float32
    e1 = np.exp(-d1 * f32(alpha)).astype(np.float32)
    e2 = np.exp(-d2 * f32(alpha)).astype(np.float32)
    losses = []
    for e, idx, n_other, frac in ((e1, i1, n_x, frac_21), (e2, i2, n_gt, frac_12)):
        cnt = np.zeros((idx.shape[0], n_other), np.int64)
        for b in range(idx.shape[0]):
            np.add.at(cnt[b], idx[b], 1)
        w = np.take_along_axis(cnt, idx.astype(np.int64), 1).astype(np.float32) ** f32(n_lambda)
        w = (f32(1) / (w + f32(1e-6))) * f32(frac)
        losses.append((f32(1) - e * w).mean(1, dtype=np.float32))
    return (losses[0] + losses[1]) / f32(2), cd_p, cd_t


def pair_rows(points, rows=None, alpha=1000):
    """points [N, n, 3] -> {i: (dcd[N-i], cd_s[N-i], cd_m[N-i])} for the requested rows
    (reference get_src_pair; float64 arrays of the fp32 values, as `.item()` gives)."""
    points = np.asarray(points, np.float32)
    n = points.shape[0]
    out = {}
    for i in (range(n) if rows is None else rows):
        xs = points[i:]
        gts = np.repeat(points[i:i + 1], n - i, axis=0)
        dcd, cd_s, cd_m = calc_dcd(xs, gts, alpha=alpha)
        out[i] = (dcd.astype(np.float64), cd_s.astype(np.float64), cd_m.astype(np.float64))
    return out


def connect_matrix(rows, n):
    """visualization.py:30-46: [3, N, N] = M + M.T of the upper-triangular rows."""
    m = np.zeros((3, n, n))
    for i, (dcd, cd_s, cd_m) in rows.items():
        m[0, i, i:], m[1, i, i:], m[2, i, i:] = dcd, cd_s, cd_m
    return m + m.transpose(0, 2, 1)
