"""Drop-in for the reference network/simple_encoder.py (TargetEncoder, STN3D).

Same constructor arguments, module attributes and state_dict keys as the
reference (network/simple_encoder.py:6-107) so checkpoints interchange; the
forward pass runs on the fused HIP chain ured_hip.mlp.PointEncoderFn.
`stn1` / `stn2` are built (their parameters are part of the checkpoint) but, as
in the reference, never called.
"""
import torch
import torch.nn as nn

from ured_hip.mlp import EncoderSpec, PointEncoderFn


def _conv_bn_relu(cin, cout):
    return [nn.Conv1d(cin, cout, 1), nn.BatchNorm1d(cout), nn.ReLU()]


def _lin_bn_relu(cin, cout):
    return [nn.Linear(cin, cout), nn.BatchNorm1d(cout), nn.ReLU()]


class STN3D(nn.Module):
    """Spatial transformer of the reference (simple_encoder.py:6-40); parameters only."""

    def __init__(self, input_channels=3):
        super().__init__()
        self.input_channels = input_channels
        self.mlp1 = nn.Sequential(*_conv_bn_relu(input_channels, 64), *_conv_bn_relu(64, 128),
                                  *_conv_bn_relu(128, 1024))
        self.mlp2 = nn.Sequential(*_lin_bn_relu(1024, 512), *_lin_bn_relu(512, 256),
                                  nn.Linear(256, input_channels * input_channels))

    def forward(self, x):
        raise NotImplementedError("STN3D is never called by U-RED (simple_encoder.py:88-107)")


class TargetEncoder(nn.Module):
    """PointNet-style per-point MLP + semantic fusion + max-pool (simple_encoder.py:43-107).

    forward(x, sem_f):
      is_src=False: x [B, N, 3], sem_f [B, N, S] -> (code [B, C], per_point [B, C, N])
      is_src=True : x [B, P, N, 3], sem_f [B, P, S] -> (code [B*P, C], per_point [B*P, C, N])
    per_point is returned as a channel-first *view* of point-major storage;
    `forward_pointmajor` returns the [rows, C] tensor itself.
    """

    def __init__(self, embedding_size=256, input_channels=3, is_src=False, sem_size=False):
        super().__init__()
        if input_channels != 3:
            raise NotImplementedError("the fused encoder handles xyz input (input_channels=3)")
        if sem_size is False:
            raise NotImplementedError("U-RED always fuses semantics (sem_size); sem_size=False is not on the path")
        self.input_channels = input_channels
        self.is_src = is_src
        self.max_part = 16
        self.sem_size = sem_size
        self.stn1 = STN3D(input_channels)
        self.stn2 = STN3D(64)
        self.mlp1 = nn.Sequential(*_conv_bn_relu(input_channels, 64), *_conv_bn_relu(64, 64))
        self.mlp2 = nn.Sequential(*_conv_bn_relu(64, 64), *_conv_bn_relu(64, 128), *_conv_bn_relu(128, 1024))
        self.fuse_sem = nn.Sequential(*_conv_bn_relu(1024 + sem_size, 1024))
        self.per_point_out = nn.Sequential(*_conv_bn_relu(1024, embedding_size)[:3],
                                           nn.Conv1d(embedding_size, embedding_size, 1))
        self.fc = nn.Linear(1024, embedding_size)
        # parity diagnostics: when set, forward keeps the max-pool winners (last_pool_idx [G, 1024])
        # and the values they were chosen from (last_pool_vals: fuse_sem's raw output [G*n, 1024] and
        # its BatchNorm scale / shift; the pooled activation is relu(y * scale + shift))
        self.record_pool = False
        self.last_pool_idx = None
        self.last_pool_vals = None

    def _layers(self):
        convs = [(self.mlp1[0], self.mlp1[1]), (self.mlp1[3], self.mlp1[4]), (self.mlp2[0], self.mlp2[1]),
                 (self.mlp2[3], self.mlp2[4]), (self.mlp2[6], self.mlp2[7]), (self.fuse_sem[0], self.fuse_sem[1]),
                 (self.per_point_out[0], self.per_point_out[1])]
        params = []
        for conv, bn in convs:
            params += [conv.weight, conv.bias, bn.weight, bn.bias]
        params += [self.per_point_out[3].weight, self.per_point_out[3].bias, self.fc.weight, self.fc.bias]
        return [bn for _, bn in convs], params

    def forward_pointmajor(self, x, sem_f, rw=None):
        """-> code [G, C], per_point [G*n, C] (point-major).

        rw: optional ured_hip.kernels.RowWeights for a unique-row batch (is_src: x holds the
        distinct source parts, rw.w[g] = how many slots of the full batch part g fills)."""
        if self.is_src:
            B, P, n, _ = x.shape
            xf = x.reshape(B * P * n, 3)
            sem = sem_f.reshape(B * P, -1)
            spec_mode = "src"
        else:
            B, n, _ = x.shape
            xf = x.reshape(B * n, 3)
            sem = sem_f.reshape(B * n, -1)
            spec_mode = "tgt"
        bns, params = self._layers()
        rec = {} if self.record_pool else None
        spec = EncoderSpec(spec_mode, n, self.training, bns, rw=rw, record=rec)
        code, pp = PointEncoderFn.apply(spec, xf.float(), sem.float(), *params)
        if rec is not None:       # the max-pool winner of every (group, channel), within its group
            G = rec["pool_rows"].shape[0]
            self.last_pool_idx = rec["pool_rows"].long() - n * torch.arange(G, device=xf.device).unsqueeze(1)
            self.last_pool_vals = (rec["pool_y"], rec["pool_scale"], rec["pool_shift"], n)
        return code, pp

    def forward(self, x, sem_f):
        n = x.shape[-2]
        code, pp = self.forward_pointmajor(x, sem_f)
        return code, pp.view(-1, n, pp.shape[-1]).permute(0, 2, 1)
