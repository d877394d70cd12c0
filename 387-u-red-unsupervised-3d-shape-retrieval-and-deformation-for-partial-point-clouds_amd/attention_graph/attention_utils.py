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

    def forward(self, x):
        for layer in self:
            if isinstance(layer, nn.Conv1d):
                x = conv1x1(layer, x)
            elif isinstance(layer, nn.ReLU):
                x = F.relu(x)
            else:
                x = layer(x)
        return x
