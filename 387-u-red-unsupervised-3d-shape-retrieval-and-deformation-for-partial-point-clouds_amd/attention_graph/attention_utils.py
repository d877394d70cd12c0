"""FeedForwardNet_norm (reference attention_graph/attention_utils.py:62-86).

A Sequential of Conv1d(k=1) -> ReLU [-> BatchNorm1d] blocks and a final Conv1d,
with the reference's module indices (so state_dict keys match).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


def conv1x1(conv, x):
    """Conv1d(k=1) on [B, Cin, n] as one matmul (hipBLASLt); MIOpen selects naive
    direct-convolution kernels for these tiny graph-node tensors (measured ~1 ms each)."""
    y = torch.matmul(conv.weight.reshape(conv.weight.shape[0], -1), x)
    return y if conv.bias is None else y + conv.bias.unsqueeze(-1)


def _ffn_layers(dims, use_norm):
    layers = []
    for cin, cout in zip(dims[:-2], dims[1:-1]):
        layers += [nn.Conv1d(cin, cout, kernel_size=1), nn.ReLU(inplace=True)]
        if use_norm == "use_bn":
            layers.append(nn.BatchNorm1d(cout))
        elif use_norm == "use_in":
            layers.append(nn.InstanceNorm1d(cout))
        elif use_norm == "use_ln":
            layers.append(nn.LayerNorm([cout, 2], elementwise_affine=True))
    layers.append(nn.Conv1d(dims[-2], dims[-1], kernel_size=1))
    return layers


class FeedForwardNet_norm(nn.Sequential):
    def __init__(self, arg_list, use_norm="use_bn"):
        super().__init__(*_ffn_layers(list(arg_list), use_norm))
        self.use_norm = use_norm

    def forward_nodes(self, x):
        """Same network on node-major x [B, n, Cin] -> [B, n, Cout]: each Conv1d(k=1) is one
        F.linear (bias fused into the GEMM), BatchNorm1d sees the [B*n, C] rows (the same
        per-channel batch statistics as on [B, C, n]); no layout copies."""
        if self.use_norm not in ("use_bn", "None", None):
            return self.forward(x.transpose(1, 2)).transpose(1, 2)
        B, n, _ = x.shape
        for layer in self:
            if isinstance(layer, nn.Conv1d):
                x = F.linear(x, layer.weight.view(layer.weight.shape[0], -1), layer.bias)
            elif isinstance(layer, nn.ReLU):
                x = F.relu(x)
            else:
                x = layer(x.reshape(B * n, -1)).view(B, n, -1)
        return x

    def forward(self, x):
        for layer in self:
            if isinstance(layer, nn.Conv1d):
                x = conv1x1(layer, x)
            elif isinstance(layer, nn.ReLU):
                x = F.relu(x)
            else:
                x = layer(x)
        return x
