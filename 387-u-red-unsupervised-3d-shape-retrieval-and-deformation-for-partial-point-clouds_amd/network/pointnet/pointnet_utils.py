"""Drop-in for the reference network/pointnet/pointnet_utils.py.

STN3d, STNkd, PointNetEncoder and feature_transform_reguliarzer with the reference's
constructor arguments, attribute names and state_dict keys (pointnet_utils.py:10-140), so
checkpoints interchange. The per-point conv stacks (Conv1d k=1 + BatchNorm1d (+ReLU)) and
their max-pools run on the fused fp32-MFMA HIP chain ured_hip.mlp.PointChainFn, point-major
[B*N, C]; the [B, C] fully-connected heads (fc1..fc3 + BatchNorm1d, a few k FLOP per cloud)
and the 3x3 / 64x64 per-cloud transforms stay torch ops on the device.

Layout: forward() takes and returns the reference's channel-first tensors; forward_pointmajor
variants take [B, N, C] and skip the transposes.
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ured_hip import kernels as K
from ured_hip.mlp import ChainSpec, PointChainFn


def _chain(convs, bns, acts, x, group_rows, training, pool=True, want_act=False):
    """Run Conv1d/BatchNorm1d pairs on point-major x [M, Cin] -> (pooled [G, C] | None, act [M, C] | None)."""
    params = []
    for c, b in zip(convs, bns):
        params += [c.weight, c.bias, b.weight, b.bias]
    spec = ChainSpec(acts, group_rows, training, list(bns), pool=pool, want_act=want_act)
    pooled, act = PointChainFn.apply(spec, x, *params)
    return (pooled if pool else None), (act if want_act else None)


class _STN(nn.Module):
    """Shared body of STN3d / STNkd (pointnet_utils.py:10-86): conv k->64->128->1024 (BN, ReLU),
    max over points, fc 1024->512->256->k*k (BN, ReLU), + identity."""

    def _transform(self, xp, k):
        B, N, C = xp.shape
        pooled, _ = _chain([self.conv1, self.conv2, self.conv3], [self.bn1, self.bn2, self.bn3],
                           [K.ACT_ENC] * 3, xp.reshape(B * N, C), N, self.training)
        x = F.relu(self.bn4(self.fc1(pooled)))
        x = F.relu(self.bn5(self.fc2(x)))
        x = self.fc3(x)
        iden = torch.eye(k, device=x.device, dtype=x.dtype).reshape(1, k * k)
        return (x + iden).view(-1, k, k)


class STN3d(_STN):
    def __init__(self, channel):
        super().__init__()
        self.conv1 = torch.nn.Conv1d(channel, 64, 1)
        self.conv2 = torch.nn.Conv1d(64, 128, 1)
        self.conv3 = torch.nn.Conv1d(128, 1024, 1)
        self.fc1 = nn.Linear(1024, 512)
        self.fc2 = nn.Linear(512, 256)
        self.fc3 = nn.Linear(256, 9)
        self.relu = nn.ReLU()
        self.bn1 = nn.BatchNorm1d(64)
        self.bn2 = nn.BatchNorm1d(128)
        self.bn3 = nn.BatchNorm1d(1024)
        self.bn4 = nn.BatchNorm1d(512)
        self.bn5 = nn.BatchNorm1d(256)

    def forward_pointmajor(self, xp):
        """xp [B, N, channel] -> trans [B, 3, 3]."""
        return self._transform(xp, 3)

    def forward(self, x):
        """x [B, channel, N] -> [B, 3, 3] (pointnet_utils.py:27-45)."""
        return self.forward_pointmajor(x.transpose(2, 1).contiguous())


class STNkd(_STN):
    def __init__(self, k=64):
        super().__init__()
        self.conv1 = torch.nn.Conv1d(k, 64, 1)
        self.conv2 = torch.nn.Conv1d(64, 128, 1)
        self.conv3 = torch.nn.Conv1d(128, 1024, 1)
        self.fc1 = nn.Linear(1024, 512)
        self.fc2 = nn.Linear(512, 256)
        self.fc3 = nn.Linear(256, k * k)
        self.relu = nn.ReLU()
        self.bn1 = nn.BatchNorm1d(64)
        self.bn2 = nn.BatchNorm1d(128)
        self.bn3 = nn.BatchNorm1d(1024)
        self.bn4 = nn.BatchNorm1d(512)
        self.bn5 = nn.BatchNorm1d(256)
        self.k = k

    def forward_pointmajor(self, xp):
        return self._transform(xp, self.k)

    def forward(self, x):
        """x [B, k, N] -> [B, k, k] (pointnet_utils.py:62-80)."""
        return self.forward_pointmajor(x.transpose(2, 1).contiguous())


class PointNetEncoder(nn.Module):
    def __init__(self, global_feat=True, feature_transform=False, channel=3):
        super().__init__()
        self.stn = STN3d(channel)
        self.conv1 = torch.nn.Conv1d(channel, 64, 1)
        self.conv2 = torch.nn.Conv1d(64, 128, 1)
        self.conv3 = torch.nn.Conv1d(128, 1024, 1)
        self.bn1 = nn.BatchNorm1d(64)
        self.bn2 = nn.BatchNorm1d(128)
        self.bn3 = nn.BatchNorm1d(1024)
        self.global_feat = global_feat
        self.feature_transform = feature_transform
        if self.feature_transform:
            self.fstn = STNkd(k=64)

    def forward_pointmajor(self, xp):
        """xp [B, N, D] -> (global feature [B, 1024], pointfeat [B, N, 64] | None, trans, trans_feat)."""
        B, N, D = xp.shape
        trans = self.stn.forward_pointmajor(xp)                       # pointnet_utils.py:105
        xt = torch.bmm(xp[:, :, :3], trans)                           # :107-111
        if D > 3:
            xt = torch.cat([xt, xp[:, :, 3:]], dim=2)
        xt = xt.reshape(B * N, D)
        tr = self.training
        if self.global_feat and not self.feature_transform:
            # conv1..conv3 as ONE fused chain (no activation is materialised)
            g, _ = _chain([self.conv1, self.conv2, self.conv3], [self.bn1, self.bn2, self.bn3],
                          [K.ACT_ENC, K.ACT_ENC, K.ACT_BN], xt, N, tr)
            return g, None, trans, None
        _, h1 = _chain([self.conv1], [self.bn1], [K.ACT_ENC], xt, N, tr, pool=False, want_act=True)   # :114
        trans_feat = None
        if self.feature_transform:                                    # :116-120
            trans_feat = self.fstn.forward_pointmajor(h1.view(B, N, 64))
            h1 = torch.bmm(h1.view(B, N, 64), trans_feat).reshape(B * N, 64)
        g, _ = _chain([self.conv2, self.conv3], [self.bn2, self.bn3], [K.ACT_ENC, K.ACT_BN], h1, N, tr)   # :124-128
        return g, h1.view(B, N, 64), trans, trans_feat

    def forward(self, x):
        """x [B, D, N] -> (x [B, 1024], trans, trans_feat) if global_feat, else
        (cat([x repeated over N, pointfeat], 1) [B, 1088, N], trans, trans_feat) (pointnet_utils.py:101-134)."""
        B, D, N = x.size()
        g, pointfeat, trans, trans_feat = self.forward_pointmajor(x.transpose(2, 1).contiguous())
        if self.global_feat:
            return g, trans, trans_feat
        gx = g.view(-1, 1024, 1).repeat(1, 1, N)
        return torch.cat([gx, pointfeat.transpose(2, 1)], 1), trans, trans_feat


def feature_transform_reguliarzer(trans):
    """mean_b || T_b T_b^T - I ||_F (pointnet_utils.py:137-141; the reference's spelling)."""
    d = trans.size()[1]
    eye = torch.eye(d, device=trans.device, dtype=trans.dtype)[None, :, :]
    return torch.mean(torch.norm(torch.bmm(trans, trans.transpose(2, 1)) - eye, dim=(1, 2)))
