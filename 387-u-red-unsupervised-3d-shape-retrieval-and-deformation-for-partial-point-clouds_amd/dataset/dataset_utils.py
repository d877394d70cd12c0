"""Drop-in for the hot-path functions of the reference dataset/dataset_utils.py.

compute_aabbox  dataset_utils.py:77-85
get_shape       dataset_utils.py:691-726   A [B,P,3n,6] @ (weight*param + default) -> [B,P,n,3]
get_source_info dataset_utils.py:791-820   (gathers from a device-resident SourceDB, no host copies)
get_source_points dataset_utils.py:1008-1034
get_symmetric   dataset_utils.py:1194-1196
get_shape_numpy dataset_utils.py:601-621    (+ deform_vertices: the same for every retrieved mesh at once)
cal_retrieval_score dataset_utils.py:1165-1176 (+ ndcg_score: sklearn.metrics.ndcg_score on the device)
The rendering / mesh export helpers of that file are out of scope; the pickle-label helpers
(get_labels, mask_label) live in train_utils/pseudo_labels.py as a device table.
"""
import numpy as np
import torch


def compute_aabbox(vertices):
    lo = vertices.min(dim=0).values
    hi = vertices.max(dim=0).values
    return torch.cat([(lo + hi) / 2.0, (hi - lo) / 2.0], dim=0)


def get_shape(A, param, src_default_param=None, weight=1.0, param_init=None, connectivity_mat=None):
    bs, num_part, pd = param.shape
    A = A.reshape(bs * num_part, -1, pd)
    p = param.reshape(bs * num_part, pd, 1)
    if param_init is not None:
        p = weight * (p - param_init.reshape(1, pd, 1))
    else:
        p = weight * p
    if src_default_param is not None:
        p = p + src_default_param.reshape(bs * num_part, pd, 1)
    if connectivity_mat is not None:
        p = torch.bmm(connectivity_mat, p)
    # A [BP, 3n, 6] @ p [BP, 6, 1] is a batched GEMV (HBM-bound: 18.9 MB of A at config 2) that the
    # BLAS libraries run as tile GEMMs (130-140 us on MI355X): one streaming HIP kernel each way
    if pd == 6 and not A.requires_grad:             # (CPU tensors raise: no fallback)
        from ured_hip.ops import GetShapeFn
        return GetShapeFn.apply(A, p.reshape(bs * num_part, pd)).reshape(bs, num_part, -1, 3)
    return torch.bmm(A, p).reshape(bs, num_part, -1, 3)


def get_shape_src(db, source_labels, param, src_default_param=None, weight=1.0):
    """get_shape(get_source_info(source_labels, db)[0], param, src_default_param, weight) — the
    training step's deformation (engine/train.py:222-223) — reading the source matrices in place:
    one HIP launch each way (ured_hip.ops.GetShapeSrcFn), no gathered [B, P, 3n, 6] copy and no
    separate parameter mul / add. Same values, bitwise."""
    bs, num_part, pd = param.shape
    if pd == 6 and param.is_cuda and not db.mats.requires_grad:
        from ured_hip.ops import GetShapeSrcFn
        labels = torch.as_tensor(source_labels, device=db.mats.device).long()
        out = GetShapeSrcFn.apply(db.mats.reshape(db.mats.shape[0], -1, pd), labels, param, src_default_param, weight)
        return out.reshape(bs, num_part, -1, 3)
    mats = get_source_info(source_labels, db, want=(True, False, False))[0]
    return get_shape(mats, param, src_default_param, weight)


_MIRROR = {}


def get_symmetric(pc):
    """x -> -x reflection (dataset_utils.py:1194-1196): the reference's multiply by [-1, 1, 1]
    (one kernel each way). The constant is made on the device by fills on first use (an H2D copy
    is not allowed inside HIP-graph capture) and cached per device and dtype."""
    key = (pc.device, pc.dtype)
    s = _MIRROR.get(key)
    if s is None:
        s = torch.ones(3, device=pc.device, dtype=pc.dtype)
        s[0] = -1.0
        _MIRROR[key] = s
    return pc * s


def _index(source_labels, db):
    idx = torch.as_tensor(source_labels, device=db.points.device).long()
    return torch.where(idx < 0, idx + db.num_sources, idx)   # python negative indexing, dataset_utils.py:800-805


def get_source_info(source_labels, db, use_connectivity=False, want=(True, True, True)):
    """-> (mats [B,P,3n,6], default_params [B,P,6], sem_idx [B,P]) gathered on the device;
    `want` skips the gathers of fields the caller does not read (None in their place)."""
    idx = _index(source_labels, db)
    return tuple(t[idx] if w else None for t, w in zip((db.mats, db.default_param, db.sem), want))


def get_source_points(source_labels, db, device=None):
    return db.points[_index(source_labels, db)]


def get_shape_numpy(A, param, src_default_param=None, weight=1.0, connectivity_mat=None):
    """dataset_utils.py:601-621 (numpy, one part): A [3V, 6] @ (weight*param + default) -> [V, 3]."""
    param = np.multiply(param, weight)
    if src_default_param is not None:
        param = param + src_default_param
    if connectivity_mat is not None:
        param = np.matmul(connectivity_mat, param)
    return np.reshape(np.matmul(A, param), (-1, 3), order="C")


def deform_vertices(vmats, voff, source_idx, params, default_params=None, weight=0.1):
    """The vis.py:291-296 mesh step for every part slot of a batch at once: part slot (b, i) uses
    the retrieved source's vertices_mat rows vmats[voff[s]:voff[s+1]] ([3V_s, 6], stacked for the
    whole source DB) and p = weight*params[b,i] + default_params[b,i] (vis.py passes the target
    part's AABB as the default). Returns (vertices [R, 3] flat over the slots in (b, i) order,
    row offsets [B*P+1]) — a ragged GEMV, HBM-bound, as device ops without a host sync except the
    output size (taken from the offsets' last entry)."""
    B, P, pd = params.shape
    src = source_idx.reshape(-1).long()
    starts, ends = voff[src].long(), voff[src + 1].long()
    counts = ends - starts                                             # rows (3 per vertex)
    out_off = torch.cat([counts.new_zeros(1), torch.cumsum(counts, 0)])
    total = int(out_off[-1])
    slot = torch.repeat_interleave(torch.arange(B * P, device=params.device), counts, output_size=total)
    row = starts[slot] + (torch.arange(total, device=params.device) - out_off[slot])
    p = weight * params.reshape(B * P, pd)
    if default_params is not None:
        p = p + default_params.reshape(B * P, pd)
    v = (vmats[row] * p[slot]).sum(-1)
    return v.view(-1, 3), torch.div(out_off, 3, rounding_mode="floor")


def ndcg_score(y_true, y_score, k=None):
    """sklearn.metrics.ndcg_score (ignore_ties=False) for each row of [Q, L] float64 tensors:
    tie-averaged DCG@k of y_true ranked by y_score over the ideal DCG@k; rows whose ideal DCG
    is 0 score 0. Returns [Q] (sklearn's value for one row is the mean over a batch of one)."""
    y_true = y_true.double()
    y_score = y_score.double()
    Q, L = y_true.shape
    disc = 1.0 / torch.log2(torch.arange(L, device=y_true.device, dtype=torch.float64) + 2.0)
    if k is not None:
        disc[k:] = 0.0
    s_sorted, order = torch.sort(y_score, dim=1, descending=True, stable=True)
    rel = torch.gather(y_true, 1, order)
    new = torch.ones_like(s_sorted, dtype=torch.bool)
    new[:, 1:] = s_sorted[:, 1:] != s_sorted[:, :-1]
    gid = torch.cumsum(new.long(), 1) - 1
    gsum = torch.zeros_like(rel).scatter_add_(1, gid, rel)
    gcnt = torch.zeros_like(rel).scatter_add_(1, gid, torch.ones_like(rel))
    dcg = (torch.gather(gsum, 1, gid) / torch.gather(gcnt, 1, gid) * disc).sum(1)
    ideal = torch.sort(y_true, dim=1, descending=True).values
    idcg = (ideal * disc).sum(1)
    return torch.where(idcg > 0, dcg / torch.where(idcg > 0, idcg, torch.ones_like(idcg)), torch.zeros_like(dcg))


def cal_retrieval_score(y_score, cd_m, k=40, sigma=0.001, aligned=False):
    """dataset_utils.py:1165-1176 for Q target parts at once: y_score [Q, NS] (cosine similarity
    of each target part to every source), cd_m [Q, NS] (the part's pseudo-label row, what
    read_pickle_topk reads) -> NDCG@k per part [Q].

    The reference builds true_relevance = exp(-d^2 / (2 sigma^2)) from read_pickle_topk's
    distances, which come back SORTED ascending (torch.topk(..., k=NS, largest=False)), and
    scores them against y_score in source order; aligned=False reproduces that, aligned=True
    scores each source's own relevance."""
    d = cd_m.double()
    if not aligned:
        d = torch.sort(d, dim=1).values
    rel = torch.exp(-d ** 2 / (2.0 * sigma ** 2))
    return ndcg_score(rel, y_score.double(), k)
