"""Drop-in for calc_cd / calc_dcd / calc_emd / fscore (Density_aware_Chamfer_Distance/utils_v2/model_utils.py:13-76,
utils_v2/metrics/CD/fscore.py) on the HIP nearest-neighbour kernels.

Note the reference's argument order: calc_cd(output, gt) evaluates cham_loss(gt, output), so
dist1 is gt -> output (model_utils.py:56); kept here.
"""
import torch

from ured_hip import nn as unn

from .dist_chamfer_3D import chamfer_3DDist


def fscore(dist1, dist2, threshold=0.0001):
    precision_1 = torch.mean((dist1 < threshold).float(), dim=1)
    precision_2 = torch.mean((dist2 < threshold).float(), dim=1)
    f = 2 * precision_1 * precision_2 / (precision_1 + precision_2)
    f[torch.isnan(f)] = 0
    return f, precision_1, precision_2


def calc_cd(output, gt, calc_f1=False, return_raw=False, normalize=False, separate=False):
    dist1, dist2, idx1, idx2 = chamfer_3DDist()(gt, output)
    cd_p = (torch.sqrt(dist1).mean(1) + torch.sqrt(dist2).mean(1)) / 2
    cd_t = dist1.mean(1) + dist2.mean(1)
    if separate:
        res = [torch.cat([torch.sqrt(dist1).mean(1).unsqueeze(0), torch.sqrt(dist2).mean(1).unsqueeze(0)]),
               torch.cat([dist1.mean(1).unsqueeze(0), dist2.mean(1).unsqueeze(0)])]
    else:
        res = [cd_p, cd_t]
    if calc_f1:
        res.append(fscore(dist1, dist2)[0])
    if return_raw:
        res.extend([dist1, dist2, idx1, idx2])
    return res


def calc_dcd(x, gt, alpha=1000, n_lambda=1, return_raw=False, non_reg=False):
    """Density-aware chamfer: 1 - exp(-alpha d) weighted by 1/(visit count of the NN) (model_utils.py:13-51)."""
    x, gt = x.float(), gt.float()
    n_x, n_gt = x.shape[1], gt.shape[1]
    if non_reg:
        frac_12, frac_21 = max(1, n_x / n_gt), max(1, n_gt / n_x)
    else:
        frac_12, frac_21 = n_x / n_gt, n_gt / n_x
    if not (torch.is_grad_enabled() and (x.requires_grad or gt.requires_grad)) and n_x + n_gt <= unn.DCD_MAX_POINTS:
        # forward-only (metrics, pseudo-labels): NN + one fused reduction kernel (ured_dcd)
        dist1, dist2, idx1, idx2 = unn.nn_dense(gt, x)
        loss, cd_p, cd_t = unn.dcd(dist1, idx1, dist2, idx2, alpha, n_lambda, frac_12, frac_21)
        res = [loss, cd_p, cd_t]
        if return_raw:
            res.extend([dist1, dist2, idx1, idx2])
        return res
    cd_p, cd_t, dist1, dist2, idx1, idx2 = calc_cd(x, gt, return_raw=True)
    # dist1/idx1: every gt point -> its NN in x; dist2/idx2: every x point -> its NN in gt
    exp1, exp2 = torch.exp(-dist1 * alpha), torch.exp(-dist2 * alpha)
    cnt1 = torch.zeros_like(idx2).scatter_add_(1, idx1.long(), torch.ones_like(idx1))
    w1 = (cnt1.gather(1, idx1.long()).float().detach() ** n_lambda + 1e-6) ** (-1) * frac_21
    loss1 = (1 - exp1 * w1).mean(dim=1)
    cnt2 = torch.zeros_like(idx1).scatter_add_(1, idx2.long(), torch.ones_like(idx2))
    w2 = (cnt2.gather(1, idx2.long()).float().detach() ** n_lambda + 1e-6) ** (-1) * frac_12
    loss2 = (1 - exp2 * w2).mean(dim=1)
    res = [(loss1 + loss2) / 2, cd_p, cd_t]
    if return_raw:
        res.extend([dist1, dist2, idx1, idx2])
    return res


def calc_emd(output, gt, eps=0.005, iterations=50):
    """utils_v2/model_utils.py:72-76: auction EMD (emdModule on csrc/emd.hip) ->
    (sqrt(dist).mean(1) [B], dist [B, n])."""
    from emd import emd
    dist, _ = emd()(output, gt, eps, iterations)
    return torch.sqrt(dist).mean(1), dist
