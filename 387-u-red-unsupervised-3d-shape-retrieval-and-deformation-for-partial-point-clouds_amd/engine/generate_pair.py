"""Offline all-pairs DCD / CD pseudo-labels on MI355X.

Drop-in for engine/generate_pair.py:69-131 (`get_src_pair`: for source part i, the
density-aware chamfer against every part j >= i, saved as a pickle
{'dcd_loss', 'cd_s', 'cd_m'} per part) and engine/visualization.py:30-46 (the [3, N, N]
`sources_connect.npy` = M + M.T of those rows).

The reference evaluates one pair per call (`compute_dcd_loss(dataset[j], dataset[i])`,
two chamfer3D launches + ~10 torch ops + 3 `.item()` syncs each, joblib over 48
processes). Here a chunk of up to `chunk_pairs` pairs is one dense NN launch
(`ured_nn_fwd`, gt = cloud i as xyz1, x = cloud j as xyz2, exactly as calc_cd calls
cham_loss(gt, output)) followed by one fused `ured_dcd` reduction; the per-pair
scalars stay in HBM until the whole shard is done (one device->host copy).

Multi-GPU: rows are independent. `shard_rows` deals them to ranks in a balanced
zig-zag (row i and row N-1-i together, so every rank gets ~the same pair count);
no collective on the data path ("weak" sharding, one process per GPU).
"""
import argparse
import os
import pickle
import sys

import numpy as np
import torch

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from ured_hip import nn as unn  # noqa: E402


def normalize_pts(pts):
    """engine/geometry_utils.py:88-94 (read_h5 normalises every part cloud)."""
    out = np.array(pts, dtype=np.float32)
    out -= np.mean(out, axis=0)
    out /= np.sqrt(np.max(np.sum(out ** 2, axis=1)))
    return out


def shard_rows(n, rank=0, world=1):
    """Rows of an N x N upper triangle for `rank`: pairs (k, N-1-k) dealt round-robin."""
    order = []
    for k in range((n + 1) // 2):
        order.append(k)
        if n - 1 - k != k:
            order.append(n - 1 - k)
    pairs = [order[i:i + 2] for i in range(0, len(order), 2)]
    return sorted(r for i, p in enumerate(pairs) if i % world == rank for r in p)


class PairGenerator:
    """All-pairs calc_dcd over a resident [N, n, 3] float32 cloud table."""

    def __init__(self, points, alpha=1000, n_lambda=1, chunk_pairs=16384):
        if points.dim() != 3 or points.shape[-1] != 3:
            raise ValueError(f"points must be [N, n, 3], got {tuple(points.shape)}")
        self.points = points.contiguous().float()
        self.alpha = alpha
        self.n_lambda = n_lambda
        self.chunk = int(min(chunk_pairs, 65535))

    def pairs(self, gi, xj, x_table=None):
        """calc_dcd(x = x_table[xj], gt = points[gi]) for index vectors (device, int64) ->
        (dcd, cd_s, cd_m) device tensors; x_table defaults to the resident table itself."""
        xt = self.points if x_table is None else x_table
        outs = []
        for s in range(0, gi.numel(), self.chunk):
            g, x = self.points[gi[s:s + self.chunk]], xt[xj[s:s + self.chunk]]
            d1, d2, i1, i2 = unn.nn_dense(g, x)
            outs.append(torch.stack(unn.dcd(d1, i1, d2, i2, self.alpha, self.n_lambda)))
        return torch.cat(outs, 1) if outs else torch.empty(3, 0, device=self.points.device)

    @torch.no_grad()
    def cross(self, targets):
        """Target parts x every resident source: calc_dcd(x = targets[t], gt = points[s]), the
        per-target-part rows the training pseudo-labels are chosen from (the target branch of
        get_data_pair, generate_pair.py:96-104: compute_dcd_loss(target part, source)).
        targets [T, n, 3] (normalised like the sources) -> [3, T, NS] device (dcd, cd_s, cd_m)."""
        targets = targets.to(self.points.device).contiguous().float()
        T, NS = targets.shape[0], self.points.shape[0]
        dev = self.points.device
        gi = torch.arange(NS, device=dev).repeat(T)
        xj = torch.arange(T, device=dev).repeat_interleave(NS)
        return self.pairs(gi, xj, targets).view(3, T, NS)

    @torch.no_grad()
    def rows(self, rows):
        """{i: (dcd[N-i], cd_s[N-i], cd_m[N-i])} float64 numpy, as get_src_pair stores them
        (`.cpu().numpy().item()` of fp32 scalars)."""
        n = self.points.shape[0]
        dev = self.points.device
        rows = list(rows)
        gi = torch.cat([torch.full((n - i,), i, dtype=torch.long) for i in rows]) if rows else torch.empty(0, dtype=torch.long)
        xj = torch.cat([torch.arange(i, n) for i in rows]) if rows else torch.empty(0, dtype=torch.long)
        res = self.pairs(gi.to(dev), xj.to(dev)).double().cpu().numpy()
        out, o = {}, 0
        for i in rows:
            out[i] = (res[0, o:o + n - i], res[1, o:o + n - i], res[2, o:o + n - i])
            o += n - i
        return out


def connect_matrix(rows, n):
    """engine/visualization.py:30-46: stack the upper-triangular rows, return M + M.T
    ([3, N, N]: dcd, cd_s, cd_m; the diagonal is counted twice, as in the reference)."""
    m = np.zeros((3, n, n))
    for i, (dcd, cd_s, cd_m) in rows.items():
        m[0, i, i:], m[1, i, i:], m[2, i, i:] = dcd, cd_s, cd_m
    return m + m.transpose(0, 2, 1)


def save_rows(out_dir, names, rows):
    """One pickle per part: {'dcd_loss', 'cd_s', 'cd_m'} (generate_pair.py:82-85)."""
    os.makedirs(out_dir, exist_ok=True)
    for i, (dcd, cd_s, cd_m) in rows.items():
        with open(os.path.join(out_dir, names[i] + ".pickle"), "wb") as f:
            pickle.dump({"dcd_loss": dcd, "cd_s": cd_s, "cd_m": cd_m}, f)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--points", help=".npy [N, n, 3] part clouds (default: synthetic source DB)")
    ap.add_argument("--num", type=int, default=512, help="synthetic: number of parts")
    ap.add_argument("--out", default="pair_out", help="directory for the per-part pickles")
    ap.add_argument("--connect", action="store_true", help="also write sources_connect.npy (rank 0, all rows)")
    ap.add_argument("--chunk", type=int, default=16384)
    a = ap.parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if a.points:
        pts = np.load(a.points, allow_pickle=False)
        pts = np.stack([normalize_pts(p) for p in pts])
    else:
        from dataset import synthetic
        pts = np.stack([normalize_pts(p) for p in synthetic.make_source_db(a.num, seed=1)["src_points"]])
    names = [f"part{i:06d}" for i in range(len(pts))]
    gen = PairGenerator(torch.from_numpy(pts).to(dev), chunk_pairs=a.chunk)
    rows = gen.rows(shard_rows(len(pts), rank, world))
    save_rows(os.path.join(a.out, "sources"), names, rows)
    if a.connect and world == 1:
        np.save(os.path.join(a.out, "sources_connect.npy"), connect_matrix(rows, len(pts)))
    print(f"rank {rank}: {len(rows)} rows, {sum(len(r[0]) for r in rows.values())} pairs -> {a.out}")


if __name__ == "__main__":
    main()
