"""Pseudo-label selection on the device: the reference's per-iteration
`get_labels` (dataset/dataset_utils.py:1101-1143) reads one pickle per target part from disk,
takes the 10 nearest sources by `cd_m` (read_pickle_topk, :1043-1051), keeps those under
`filter_threshold`, prefers one with the part's semantic label, and then drops (-1) every
later part of the sample whose choice is mutually among the `cl_k` nearest sources of an
earlier part's choice (mask_label / check_similarity, :1070-1086, on the sources_connect
distance matrix). ("TODO: Do not read file in training", :1100.)

Here the table of target-part x source distances is loaded ONCE into HBM — straight from
PairGenerator.cross (engine/generate_pair.py) or from the per-part pickles it writes — and a
batch's labels are a handful of device ops (sort, gather, first-true selection, one lookup in
a precomputed [NS, NS] mutual-top-k matrix): no file reads, no host sync.

Tie rules (the reference leaves them to torch.topk / np.argpartition): candidates are ordered
by (distance, source index), so equal distances go to the lower source index, and the `cl_k`
nearest sources of a row are the first `cl_k` in that order.
"""
import os
import pickle

import numpy as np
import torch


class PseudoLabelTable:
    """cd_m [T, NS] (target part x source, float64 as the pickles hold it), part_sem [T]
    (semantic id of each target part), sources_sem [NS], dist_src [NS, NS]."""

    def __init__(self, cd_m, part_sem, sources_sem, dist_src, alpha=2e-2, cl_k=40, topk=10, device=None):
        dev = torch.device(device) if device is not None else torch.as_tensor(cd_m).device
        self.cd_m = torch.as_tensor(cd_m, dtype=torch.float64).to(dev).contiguous()
        self.part_sem = torch.as_tensor(part_sem, dtype=torch.int64).to(dev)
        self.sources_sem = torch.as_tensor(sources_sem, dtype=torch.int64).to(dev)
        T, NS = self.cd_m.shape
        if self.part_sem.shape != (T,) or self.sources_sem.shape != (NS,):
            raise ValueError("part_sem must be [T] and sources_sem [NS] for a [T, NS] table")
        d = torch.as_tensor(dist_src, dtype=torch.float64).to(dev)
        if d.shape != (NS, NS):
            raise ValueError(f"dist_src must be [{NS}, {NS}], got {tuple(d.shape)}")
        self.alpha, self.cl_k, self.topk = float(alpha), int(cl_k), int(topk)
        self.mutual = self._mutual_topk(d, self.cl_k)
        self.device = dev

    @staticmethod
    def _order(v):
        """Indices of v's last dim sorted by (value, index)."""
        return torch.sort(v, dim=-1, stable=True).indices

    @classmethod
    def _mutual_topk(cls, d, k):
        """mutual[a, b] = b among the k nearest of a AND a among the k nearest of b
        (check_similarity, dataset_utils.py:1070-1075)."""
        NS = d.shape[0]
        k = min(k, NS)
        near = torch.zeros(NS, NS, dtype=torch.bool, device=d.device)
        near.scatter_(1, cls._order(d)[:, :k], True)
        return near & near.t()

    @classmethod
    def from_pickles(cls, pickle_dir, part_names, part_sem, sources_sem, dist_src, **kw):
        """Rows from the per-part pickles {'dcd_loss','cd_s','cd_m'} (generate_pair.py:82-85;
        our own engine/generate_pair.save_rows writes the same)."""
        rows = []
        for name in part_names:
            with open(os.path.join(pickle_dir, name + ".pickle"), "rb") as f:
                rows.append(np.asarray(pickle.load(f)["cd_m"], dtype=np.float64))
        return cls(np.stack(rows), part_sem, sources_sem, dist_src, **kw)

    def labels(self, part_rows):
        """part_rows [B, P] int (table row of each target part, -1 for absent slots; the
        present parts of a sample come first, as get_labels fills source_labels[j, :k]) ->
        source_labels [B, P] int64 (-1: absent or masked part)."""
        part_rows = torch.as_tensor(part_rows, device=self.device).long()
        present = part_rows >= 0
        rows = part_rows.clamp(min=0)
        cd = self.cd_m[rows]                                              # [B, P, NS]
        cand = self._order(cd)[..., :self.topk]                           # [B, P, K]
        dist = torch.gather(cd, -1, cand)
        ok_d = dist < self.alpha
        ok_s = ok_d & (self.sources_sem[cand] == self.part_sem[rows].unsqueeze(-1))
        K = cand.shape[-1]
        pos = torch.arange(K, device=self.device)

        def first(mask):                                                  # first True position, K if none
            return torch.where(mask, pos, torch.full_like(pos, K)).amin(-1)
        fs, fd = first(ok_s), first(ok_d)
        pick = torch.where(fs < K, fs, torch.where(fd < K, fd, torch.zeros_like(fd)))
        lab = torch.gather(cand, -1, pick.unsqueeze(-1)).squeeze(-1)      # [B, P]
        # mask_label: part j dropped if an earlier part i < j has a mutually-near choice
        P = lab.shape[1]
        sim = self.mutual[lab.unsqueeze(2), lab.unsqueeze(1)]             # [B, i, j]
        earlier = torch.triu(torch.ones(P, P, dtype=torch.bool, device=self.device), diagonal=1)
        both = present.unsqueeze(2) & present.unsqueeze(1)
        masked = (sim & earlier & both).any(1)
        return torch.where(present & ~masked, lab, torch.full_like(lab, -1))
