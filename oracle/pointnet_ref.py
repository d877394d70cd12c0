"""CPU restatement of the reference PointNetEncoder — TEST INFRASTRUCTURE ONLY.

Functional torch-CPU (float64 or float32) form over state_dict-keyed parameters of
  STN3d.forward            network/pointnet/pointnet_utils.py:27-45
  STNkd.forward            network/pointnet/pointnet_utils.py:62-80
  PointNetEncoder.forward  network/pointnet/pointnet_utils.py:101-134
  feature_transform_reguliarzer  :135-141
BatchNorm in training mode (batch statistics, biased variance for normalisation) as
torch.nn.BatchNorm1d. Pinned against tests/golden/pointnet.npz, produced by the reference
module itself (tests/golden/make_golden_pointnet.py).
"""
import numpy as np
import torch
import torch.nn.functional as F

EPS = 1e-5


def pointnet_keys(channel=3, feature_transform=False):
    """(key, shape) list of PointNetEncoder(channel, feature_transform).state_dict() (float entries)."""
    def stn(prefix, k_in, k_out):
        out = [(f"{prefix}conv1.weight", (64, k_in, 1)), (f"{prefix}conv1.bias", (64,)),
               (f"{prefix}conv2.weight", (128, 64, 1)), (f"{prefix}conv2.bias", (128,)),
               (f"{prefix}conv3.weight", (1024, 128, 1)), (f"{prefix}conv3.bias", (1024,)),
               (f"{prefix}fc1.weight", (512, 1024)), (f"{prefix}fc1.bias", (512,)),
               (f"{prefix}fc2.weight", (256, 512)), (f"{prefix}fc2.bias", (256,)),
               (f"{prefix}fc3.weight", (k_out, 256)), (f"{prefix}fc3.bias", (k_out,))]
        for i, c in ((1, 64), (2, 128), (3, 1024), (4, 512), (5, 256)):
            out += _bn(f"{prefix}bn{i}.", c)
        return out
    keys = stn("stn.", channel, 9)
    keys += [("conv1.weight", (64, channel, 1)), ("conv1.bias", (64,)), ("conv2.weight", (128, 64, 1)),
             ("conv2.bias", (128,)), ("conv3.weight", (1024, 128, 1)), ("conv3.bias", (1024,))]
    for i, c in ((1, 64), (2, 128), (3, 1024)):
        keys += _bn(f"bn{i}.", c)
    if feature_transform:
        keys += stn("fstn.", 64, 64 * 64)
    return keys


def _bn(prefix, c):
    return [(prefix + "weight", (c,)), (prefix + "bias", (c,)), (prefix + "running_mean", (c,)),
            (prefix + "running_var", (c,))]


def make_params(channel=3, feature_transform=False, seed=0):
    """Deterministic parameters (numpy PCG64): conv/fc weights U(+-1/sqrt(fan_in)), biases
    U(+-0.1), BN gamma U(-0.4, 1.6) (some negative: exercises the min side of the max-pool),
    beta U(+-0.2), running stats (0, 1). Returns the full state_dict {key: tensor}."""
    rng = np.random.Generator(np.random.PCG64(seed))
    P = {}
    for k, shp in pointnet_keys(channel, feature_transform):
        if k.endswith("running_mean"):
            v = np.zeros(shp)
        elif k.endswith("running_var"):
            v = np.ones(shp)
        elif ".bn" in "." + k and k.endswith("weight"):
            v = rng.uniform(-0.4, 1.6, shp)
        elif ".bn" in "." + k and k.endswith("bias"):
            v = rng.uniform(-0.2, 0.2, shp)
        elif k.endswith("weight"):
            v = rng.uniform(-1.0, 1.0, shp) / np.sqrt(shp[1] * (shp[2] if len(shp) > 2 else 1))
        else:
            v = rng.uniform(-0.1, 0.1, shp)
        P[k] = torch.from_numpy(v.astype(np.float32))
        if k.endswith("running_var"):
            P[k[:-len("running_var")] + "num_batches_tracked"] = torch.zeros((), dtype=torch.long)
    return P


def _bn_train(x, P, prefix):
    """BatchNorm1d (training) on [B, C] or [B, C, N]."""
    return F.batch_norm(x, None, None, P[prefix + "weight"], P[prefix + "bias"], training=True, eps=EPS)


def _conv(x, P, name):
    return F.conv1d(x, P[name + ".weight"], P[name + ".bias"])


def stn_forward(P, x, prefix, k):
    """STN3d / STNkd forward (pointnet_utils.py:27-45 / 62-80): x [B, C, N] -> [B, k, k]."""
    B = x.shape[0]
    x = F.relu(_bn_train(_conv(x, P, prefix + "conv1"), P, prefix + "bn1."))
    x = F.relu(_bn_train(_conv(x, P, prefix + "conv2"), P, prefix + "bn2."))
    x = F.relu(_bn_train(_conv(x, P, prefix + "conv3"), P, prefix + "bn3."))
    x = torch.max(x, 2, keepdim=True)[0].view(-1, 1024)
    x = F.relu(_bn_train(F.linear(x, P[prefix + "fc1.weight"], P[prefix + "fc1.bias"]), P, prefix + "bn4."))
    x = F.relu(_bn_train(F.linear(x, P[prefix + "fc2.weight"], P[prefix + "fc2.bias"]), P, prefix + "bn5."))
    x = F.linear(x, P[prefix + "fc3.weight"], P[prefix + "fc3.bias"])
    iden = torch.eye(k, dtype=x.dtype).reshape(1, k * k).repeat(B, 1)
    return (x + iden).view(-1, k, k)


def pointnet_forward(P, x, global_feat=True, feature_transform=False):
    """PointNetEncoder.forward (pointnet_utils.py:101-134): x [B, D, N] -> (out, trans, trans_feat)."""
    B, D, N = x.size()
    trans = stn_forward(P, x, "stn.", 3)
    x = x.transpose(2, 1)
    if D > 3:
        feature = x[:, :, 3:]
        x = x[:, :, :3]
    x = torch.bmm(x, trans)
    if D > 3:
        x = torch.cat([x, feature], dim=2)
    x = x.transpose(2, 1)
    x = F.relu(_bn_train(_conv(x, P, "conv1"), P, "bn1."))
    trans_feat = None
    if feature_transform:
        trans_feat = stn_forward(P, x, "fstn.", 64)
        x = torch.bmm(x.transpose(2, 1), trans_feat).transpose(2, 1)
    pointfeat = x
    x = F.relu(_bn_train(_conv(x, P, "conv2"), P, "bn2."))
    x = _bn_train(_conv(x, P, "conv3"), P, "bn3.")
    x = torch.max(x, 2, keepdim=True)[0].view(-1, 1024)
    if global_feat:
        return x, trans, trans_feat
    x = x.view(-1, 1024, 1).repeat(1, 1, N)
    return torch.cat([x, pointfeat], 1), trans, trans_feat


def feature_transform_reguliarzer(trans):
    d = trans.size()[1]
    eye = torch.eye(d, dtype=trans.dtype, device=trans.device)[None, :, :]
    return torch.mean(torch.norm(torch.bmm(trans, trans.transpose(2, 1)) - eye, dim=(1, 2)))


CASES = [  # (name, B, D, N, global_feat, feature_transform)
    ("g_n256", 4, 3, 256, True, False),
    ("l_ft_n200", 3, 3, 200, False, True),
    ("g_d6_n128", 2, 6, 128, True, False),
]


def case_inputs(B, D, N, seed):
    """Seeded inputs: points x [B, D, N] and the loss weights R for (out, trans, trans_feat)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    x = rng.uniform(-1, 1, (B, D, N)).astype(np.float32)
    return x, rng


def case_loss(out, trans, trans_feat, rng_seed):
    """Scalar loss sum(out*R1) + sum(trans*R2) (+ sum(trans_feat*R3) + regulariser), R seeded."""
    g = torch.Generator().manual_seed(rng_seed)
    loss = (out * torch.randn(out.shape, generator=g).to(out)).sum()
    loss = loss + (trans * torch.randn(trans.shape, generator=g).to(trans)).sum()
    if trans_feat is not None:
        loss = loss + (trans_feat * torch.randn(trans_feat.shape, generator=g).to(trans_feat)).sum()
        loss = loss + feature_transform_reguliarzer(trans_feat)
    return loss
