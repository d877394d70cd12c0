"""Drop-in for the hot-path functions of the reference dataset/dataset_utils.py.

compute_aabbox  dataset_utils.py:77-85
get_shape       dataset_utils.py:691-726   A [B,P,3n,6] @ (weight*param + default) -> [B,P,n,3]
get_source_info dataset_utils.py:791-820   (gathers from a device-resident SourceDB, no host copies)
get_source_points dataset_utils.py:1008-1034
get_symmetric   dataset_utils.py:1194-1196
The rendering / mesh export / pickle-label helpers of that file are out of scope.
"""
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
    return torch.bmm(A, p).reshape(bs, num_part, -1, 3)


def get_symmetric(pc):
    """x -> -x reflection (dataset_utils.py:1194-1196). Built without a host-made constant
    tensor (an H2D copy is not allowed inside HIP-graph capture); negation is exact, so the
    values equal the reference's multiply by [-1, 1, 1]."""
    return torch.cat((-pc[..., :1], pc[..., 1:]), dim=-1)


def _index(source_labels, db):
    idx = torch.as_tensor(source_labels, device=db.points.device).long()
    return torch.where(idx < 0, idx + db.num_sources, idx)   # python negative indexing, dataset_utils.py:800-805


def get_source_info(source_labels, db, use_connectivity=False):
    """-> (mats [B,P,3n,6], default_params [B,P,6], sem_idx [B,P]) gathered on the device."""
    idx = _index(source_labels, db)
    return db.mats[idx], db.default_param[idx], db.sem[idx]


def get_source_points(source_labels, db, device=None):
    return db.points[_index(source_labels, db)]
