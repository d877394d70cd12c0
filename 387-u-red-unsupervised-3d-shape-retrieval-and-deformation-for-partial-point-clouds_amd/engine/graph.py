"""The training step as HIP graphs (torch.cuda.CUDAGraph = hipGraph on ROCm).

One eager step issues ~1400 kernel launches (the fused HIP GEMMs plus many small torch ops of
DeformNet, the losses and the optimizer); their host-side launch cost leaves the GPU idle for
several ms per step. The step has static shapes and no host sync (segment tables and part
pooling are built on device), so it is captured once and replayed:

  graph 1: zero_grad + forward + backward      (our ctypes launches go to torch's current
                                                 stream, i.e. the capture stream)
  eager  : reduce_gradients()                   (RCCL bucketed all-reduce when world > 1)
  graph 2: clip_grad_norm_ x6 + Adam            (Adam built with capturable=True)

Inputs are copied into static buffers before each replay; the returned loss dict holds the
graph's static output tensors (valid until the next replay). Same kernels, same arithmetic
as the eager step: a replay is bit-identical to an eager step on the same state and batch.
With world > 1 the forward contains the contrastive loss's all_gather; graph mode is then
opt-in (cfg["cuda_graph_dp"]), the default keeps the eager path.
"""
import torch


class GraphedStep:
    def __init__(self, inner, example_batch, warmup=3):
        self.inner = inner
        # tensors only: a UniqueRows entry (data-dependent shapes) cannot live in static buffers,
        # so the graphed step encodes every source slot
        self.static = {k: v.clone() for k, v in example_batch.items() if torch.is_tensor(v)}
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):   # warm-up: library loads, allocator, hipBLASLt workspaces
            for _ in range(warmup):
                inner.step(self.static)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.pool = torch.cuda.graph_pool_handle()
        self.g_fwd_bwd = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_fwd_bwd, pool=self.pool):
            inner.optimizer.zero_grad(set_to_none=True)
            loss, self.T = inner.forward(self.static)
            loss.backward()
        self.g_update = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_update, pool=self.pool):
            inner.clip_and_step()

    @property
    def models(self):
        return self.inner.models

    @property
    def optimizer(self):
        return self.inner.optimizer

    def step(self, batch, epoch=0):
        for k, v in self.static.items():
            v.copy_(batch[k], non_blocking=True)
        self.g_fwd_bwd.replay()
        self.inner.reduce_gradients()
        self.g_update.replay()
        return self.T
