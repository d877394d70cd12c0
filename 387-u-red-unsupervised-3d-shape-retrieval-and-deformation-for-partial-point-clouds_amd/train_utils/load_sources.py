"""Source-part database (reference train_utils/load_sources.py:8-62), device resident.

The reference loads one h5 per source part (points[1024,3], points_mat[3072,6],
default_param[6], semantic label, mesh) into a list of dicts plus the
sources_connect.npy distance matrix (`dist_src`, load_sources.py:13: [3, NS, NS] = dcd, cd_s,
cd_m of every source pair, engine/visualization.py:30-46). Here the arrays live in HBM as
stacked tensors (SourceDB) so the per-step gathers are device ops. With cfg["synthetic"]
the arrays come from dataset.synthetic.make_source_db. `dist_src` is read from
cfg["src_connectivity"] when that .npy exists (np.load without pickles); otherwise it is
computed on the device from the source clouds by the same all-pairs calc_dcd as the
reference's offline generator (engine/generate_pair.py PairGenerator + connect_matrix).
"""
import os

import numpy as np
import torch

from dataset import synthetic


class SourceDB:
    def __init__(self, points, mats, default_param, sem, device):
        self.points = torch.as_tensor(points, dtype=torch.float32).to(device).contiguous()
        self.mats = torch.as_tensor(mats, dtype=torch.float32).to(device).contiguous()
        self.default_param = torch.as_tensor(default_param, dtype=torch.float32).to(device).contiguous()
        self.sem = torch.as_tensor(sem, dtype=torch.int64).to(device).contiguous()
        self.num_sources = self.points.shape[0]

    def __len__(self):
        return self.num_sources


def load_sources(cfg, device=None):
    device = device or cfg.get("device", "cuda")
    if not cfg.get("synthetic", True):
        raise NotImplementedError("on-disk PartNet h5 loading is out of scope this round; set \"synthetic\": true")
    n = int(cfg.get("num_source", -1))
    n = 512 if n <= 0 else n
    d = synthetic.make_source_db(n, seed=int(cfg.get("seed", 0)) + 1)
    db = SourceDB(d["src_points"], d["src_mats"], d["src_default_param"], d["src_sem"], device)
    path = cfg.get("src_connectivity")
    if path and os.path.exists(path):
        dist_src = np.load(path, allow_pickle=False)
        if dist_src.shape != (3, n, n):
            raise ValueError(f"{path}: expected [3, {n}, {n}], got {dist_src.shape}")
    elif cfg.get("compute_connectivity", True) and torch.device(device).type == "cuda":
        dist_src = source_connectivity(db)
    else:
        dist_src = np.zeros((3, n, n), np.float64)
    return db, dist_src


def source_connectivity(db):
    """[3, NS, NS] (dcd, cd_s, cd_m) of every pair of normalised source clouds: the reference's
    sources_connect.npy (generate_pair.get_src_pair rows + visualization.py:30-46)."""
    from engine.generate_pair import PairGenerator, connect_matrix, normalize_pts
    pts = np.stack([normalize_pts(p) for p in db.points.cpu().numpy()])
    gen = PairGenerator(torch.from_numpy(pts).to(db.points.device))
    return connect_matrix(gen.rows(range(db.num_sources)), db.num_sources)
