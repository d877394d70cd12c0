"""Drop-in for the reference network/deformation_net.py (DeformNet_MatchingNet, re_residual_net).

State-dict keys and constructor arguments follow the reference
(network/deformation_net.py:43-107). re_residual_net runs on the fused HIP chain
ured_hip.mlp.ResidualNetFn; DeformNet_MatchingNet (2 + MAX_NUM_PARTS graph nodes per sample)
runs its graph attention and param_decoder on the node kernels of csrc/node.hip
(ured_hip.node) and csrc/attn.hip.
"""
import torch
import torch.nn as nn

from attention_graph.attention_gnn import GraphAttentionNet
from attention_graph.attention_utils import FeedForwardNet_norm
from ured_hip.mlp import ResidualNetFn
from ured_hip.node import param_decoder as node_param_decoder


class DeformNet_MatchingNet(nn.Module):
    """Graph attention over [mean source part, target] global nodes and the source part
    nodes, then param_decoder -> per-part box deltas [B, P, 6] (deformation_net.py:74-93)."""

    def __init__(self, input_dim, num_stages=2, num_heads=4, part_latent_dim=256,
                 graph_dim=128, output_dim=6, use_offset=False, point_f_dim=256,
                 points_num=2048, max_num_parts=12, matching=True):
        super().__init__()
        self.input_dim = input_dim
        self.num_stages = num_stages
        self.num_heads = num_heads
        self.use_offset = use_offset
        self.output_dim = output_dim
        self.graph_dim = graph_dim
        self.point_f_dim = point_f_dim
        self.points_num = points_num
        self.max_num_parts = max_num_parts
        self.part_encoding = FeedForwardNet_norm([part_latent_dim, 128, graph_dim], use_norm="None")  # unused
        self.param_decoder = FeedForwardNet_norm([input_dim, 256, output_dim], use_norm="None")
        self.graph_attention_net = GraphAttentionNet(num_stages, graph_dim, num_heads, use_offset=use_offset)
        self.matching = matching
        self.matching_net = (FeedForwardNet_norm([point_f_dim + graph_dim * 2, 512, 1024, points_num], use_norm="use_bn")
                             if matching else None)

    def forward(self, target_f, src_part_f, per_point_f=None):
        """Node-major throughout: the reference's [B, C, nodes] tensors are held as [B, nodes, C]
        (same values; channel-first views are never materialised)."""
        bs = target_f.shape[0]
        parts = src_part_f.reshape(bs, src_part_f.shape[1], -1)                        # [B, P, C]
        nodes = torch.stack([parts.mean(dim=1), target_f], dim=1)                      # [B, 2, C]
        nodes, parts = self.graph_attention_net.forward_nodes(nodes, parts)
        P = parts.shape[1]
        if self.param_decoder.use_norm in ("None", None) and len(self.param_decoder) == 3:
            # cat([g0 | g1 broadcast to the parts, parts]): the global half as a per-sample row bias
            out = node_param_decoder(self.param_decoder, nodes.reshape(bs, -1), parts.reshape(bs * P, -1), P)
            return out.view(bs, P, -1)
        glob = nodes.reshape(bs, 1, -1).expand(-1, P, -1)                              # [g0 | g1] per part
        return self.param_decoder.forward_nodes(torch.cat([glob, parts], dim=-1))      # [B, P, 6]


class re_residual_net(nn.Module):
    """Per-point MLP in -> 256 -> 256 -> 32 -> 3 (Conv -> ReLU -> BN), deformation_net.py:96-107."""

    def __init__(self, input_dim, output_dim=3):
        super().__init__()
        self.input_dim = input_dim
        self.residual_net = FeedForwardNet_norm([input_dim, 256, 256, 32, output_dim], use_norm="use_bn")

    def _params(self):
        s = self.residual_net
        return [s[0].weight, s[0].bias, s[2].weight, s[2].bias, s[3].weight, s[3].bias, s[5].weight, s[5].bias,
                s[6].weight, s[6].bias, s[8].weight, s[8].bias, s[9].weight, s[9].bias], [s[2], s[5], s[8]]

    def forward_split(self, pp, code, *, code_first=False, group_rows=0, gidx=None, off=None, rw=None):
        """Fused form of forward(cat(pp, code[group(row)])) (or cat(code, pp) if code_first).

        pp [M, Cp] point-major, code [G, Cc]; rows grouped by fixed group_rows or by
        gidx (int32 [M]) + off (int32 [G+1], rows of group g = off[g]..off[g+1]).
        rw: optional ured_hip.kernels.RowWeights (unique-row batch, see ResidualNetFn).
        """
        params, bns = self._params()
        spec = (code_first, gidx, off, group_rows, self.training, bns, rw)
        return ResidualNetFn.apply(spec, pp, code, *params)

    def forward(self, concat_feature):
        assert self.input_dim == concat_feature.shape[-1]
        B, N, Cin = concat_feature.shape
        flat = concat_feature.reshape(B * N, Cin)
        empty_code = flat.new_zeros(1, 0)
        out = self.forward_split(flat, empty_code, group_rows=B * N)
        return out.view(B, N, -1)
