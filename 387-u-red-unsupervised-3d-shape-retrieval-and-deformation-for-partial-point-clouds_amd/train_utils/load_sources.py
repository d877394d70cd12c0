"""Source-part database (reference train_utils/load_sources.py:8-62), device resident.

The reference loads one h5 per source part (points[1024,3], points_mat[3072,6],
default_param[6], semantic label, mesh) into a list of dicts plus the
cfg["src_connectivity"] matrix `dist_src` (load_sources.py:13, a plain np.load). `dist_src` is
consumed only by get_labels -> mask_label -> check_similarity, which takes a ROW per source
label (`dist_src[label]`, dataset/dataset_utils.py:1070-1075): a 2-D [NS, NS] distance matrix.
engine/visualization.py:30-46 writes the [3, NS, NS] stack (dcd, cd_s, cd_m) of every source
pair; when such a stack is given, its cd_m plane ([2]) is the matrix used (the distance the
pseudo-labels themselves are ranked by, dataset_utils.py:1047).

Here the arrays live in HBM as stacked tensors (SourceDB) so the per-step gathers are device
ops. With cfg["synthetic"] the arrays come from dataset.synthetic.make_source_db. `dist_src`
(returned 2-D [NS, NS]) is read from cfg["src_connectivity"] when that .npy exists (np.load
without pickles); otherwise it is computed on the device from the source clouds by the same
all-pairs calc_dcd as the reference's offline generator (engine/generate_pair.py
PairGenerator + connect_matrix, cd_m plane).
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


def connectivity_matrix(arr, n, where="dist_src", plane=2):
    """The [NS, NS] matrix get_labels rows are taken from: a 2-D [n, n] array as is, plane `plane`
    (cfg["src_connectivity_plane"], default 2 = cd_m) of a [3, n, n] (dcd, cd_s, cd_m)
    sources_connect stack; anything else raises. The reference indexes dist_src[label] of
    whatever array its file holds; no reference file or fixture says which plane that is, so the
    default is an assumption (the plane PairGenerator writes as M + M.T of cd_m)."""
    arr = np.asarray(arr)
    if arr.shape == (n, n):
        return arr
    if arr.shape == (3, n, n):
        if plane not in (0, 1, 2):
            raise ValueError(f"{where}: src_connectivity_plane must be 0 (dcd), 1 (cd_s) or 2 (cd_m), got {plane}")
        return arr[plane]
    raise ValueError(f"{where}: expected [{n}, {n}] (or a [3, {n}, {n}] dcd/cd_s/cd_m stack), got {arr.shape}")


def load_sources(cfg, device=None):
    device = device or cfg.get("device", "cuda")
    if not cfg.get("synthetic", True):
        raise NotImplementedError("on-disk PartNet h5 loading is out of scope (h5py is not in this image); "
                                  "set \"synthetic\": true")
    n = int(cfg.get("num_source", -1))
    n = 512 if n <= 0 else n
    d = synthetic.make_source_db(n, seed=int(cfg.get("seed", 0)) + 1)
    db = SourceDB(d["src_points"], d["src_mats"], d["src_default_param"], d["src_sem"], device)
    path = cfg.get("src_connectivity")
    if path and os.path.exists(path):
        dist_src = connectivity_matrix(np.load(path, allow_pickle=False), n, where=path,
                                       plane=int(cfg.get("src_connectivity_plane", 2)))
    elif cfg.get("compute_connectivity", True) and torch.device(device).type == "cuda":
        dist_src = source_connectivity(db)[int(cfg.get("src_connectivity_plane", 2))]
    else:
        dist_src = np.zeros((n, n), np.float64)
    return db, dist_src


def source_connectivity(db):
    """[3, NS, NS] (dcd, cd_s, cd_m) of every pair of normalised source clouds: the reference's
    sources_connect.npy (generate_pair.get_src_pair rows + visualization.py:30-46)."""
    from engine.generate_pair import PairGenerator, connect_matrix, normalize_pts
    pts = np.stack([normalize_pts(p) for p in db.points.cpu().numpy()])
    gen = PairGenerator(torch.from_numpy(pts).to(db.points.device))
    return connect_matrix(gen.rows(range(db.num_sources)), db.num_sources)
