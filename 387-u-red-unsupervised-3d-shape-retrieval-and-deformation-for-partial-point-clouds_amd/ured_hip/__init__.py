"""ured_hip — the MI355X (gfx950) hot path of U-RED on libured_hip.so.

  _lib     ctypes loader of the C-ABI (include/ured_hip.h); raises if missing
  nn       nearest-neighbour / chamfer autograd ops (dense + ragged segments)
  kernels  typed wrappers of the fused per-point MLP entry points
  mlp      PointEncoderFn / ResidualNetFn autograd chains
  attn     graph-node multi-head attention (DeformNet's GraphAttentionNet core)
  optim    FlatAdam: per-module gradient clipping + Adam over flat buffers
  node     DeformNet graph-node GEMM / BatchNorm launches
  ops      device-side part building (segment sums, AABBs)
  losshead the step's loss head (chamfer families, contrastive, residual, reconstruction, weighted sum)
"""
from . import _lib, attn, kernels, losshead, nn, node, ops, optim, syncbn  # noqa: F401
