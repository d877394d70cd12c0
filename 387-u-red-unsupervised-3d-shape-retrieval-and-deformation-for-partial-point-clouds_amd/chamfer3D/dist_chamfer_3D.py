"""Drop-in for Density_aware_Chamfer_Distance/utils_v2/metrics/CD/chamfer3D/dist_chamfer_3D.py.

chamfer_3DDist()(xyz1 [b,n,3], xyz2 [b,m,3]) -> (dist1 [b,n], dist2 [b,m], idx1 [b,n] int32, idx2 [b,m] int32),
squared distances, lowest index on ties, GPU tensors only — as the reference
(dist_chamfer_3D.py:26-74), on the HIP kernels of libured_hip.so instead of a JIT-built
CUDA extension. The backward is deterministic (no float atomics, chamfer3D.cu:166-171).
"""
import torch.nn as nn

from ured_hip.nn import NNDenseFunction

chamfer_3DFunction = NNDenseFunction


class chamfer_3DDist(nn.Module):
    def forward(self, input1, input2):
        return NNDenseFunction.apply(input1.contiguous(), input2.contiguous())
