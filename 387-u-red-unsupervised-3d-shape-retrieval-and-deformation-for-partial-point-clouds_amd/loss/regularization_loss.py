"""Drop-in for the reference loss/regularization_loss.py:49-53 (regularization_param).

The only function of that module the training step calls (engine/train.py:281-283, behind
cfg["use_param_loss"] > 0). The reference boolean-indexes params_full by mask_part, which
needs a host sync for the row count; here the masked mean is taken as
sum(mask * |p|_2) / sum(mask) over all B*P rows — the same value (the unmasked rows contribute
0 and get a 0 gradient), no sync, four small launches. The rest of the reference module
(regularization_m*, regularization_re_residuals) is not called by any engine script.
"""
import torch


def regularization_param(params_full, mask_part):
    """params_full [B, P, 6] (DeformNet output), mask_part [B, P] (1 = valid part slot)
    -> mean over valid slots of the L2 norm of the slot's 6 deformation parameters."""
    m = mask_part.reshape(-1).to(params_full.dtype)
    norms = torch.linalg.vector_norm(params_full.reshape(-1, 6), ord=2, dim=-1)
    return (norms * m).sum() / m.sum()
