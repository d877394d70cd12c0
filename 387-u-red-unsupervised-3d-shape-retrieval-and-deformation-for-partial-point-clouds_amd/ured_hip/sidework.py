"""Weight-gradient work of the per-point chains on a second HIP stream.

In the backward of a Conv1d+BN chain (PointEncoderFn, ResidualNetFn) only the input-gradient
chain is sequential: dgrad -> BN-backward finalize -> BN-backward apply -> next dgrad. The
weight gradient of each layer (split-K wgrad + its reduce) and the bias column sums read the
layer's dY and nothing downstream reads them until the optimizer. Forked onto a side stream they
run beside the chain: the HBM-bound BN-backward apply and the latency-bound finalizes / column
sums of the chain share the CUs with the MFMA-bound wgrad, and each GEMM's last partial round of
tiles is filled by the other stream's blocks.

Every fork waits for everything the main stream issued so far (so a fork sees its inputs), the
tensors a fork reads are kept referenced until join(), and join() makes the main stream wait for
the side stream before the Function returns its gradients to autograd. Results are bitwise those
of the one-stream order: each kernel computes the same values, in a fixed order of its own,
whatever runs beside it. Works under HIP-graph capture (fork / join become graph edges).

URED_WGRAD_STREAM selects what goes to the side stream: 0 nothing (one stream), 1 the weight
gradients whole (wgrad GEMMs too), 2 only the short kernels behind them (split-K reduces,
bias / group column sums, the skinny edge-layer wgrads) while the wgrad GEMMs stay in order on
the main stream.

Measured slower on MI355X in graph replay (config-2 step, same-box A/B, 3 reps each, tools/
gpu_ab_multi.sh): one stream 66.3 it/s, mode 1 65.5, mode 2 63.4. The wgrad GEMMs already fill
the chip (two MFMA-bound GEMMs side by side only share it, and thrash each XCD's L2), and each
fork / join is a cross-stream graph edge whose wait costs more than the few-microsecond kernels
it lets overlap. Default 0; the mechanism stays for other shapes / hardware (bitwise-tested).
"""
import os

import torch

MODE = int(os.environ.get("URED_WGRAD_STREAM", "0"))
_SIDE = {}


def _side_stream(dev):
    s = _SIDE.get(dev.index)
    if s is None:
        s = _SIDE[dev.index] = torch.cuda.Stream(device=dev)
    return s


class SideWork:
    """big(fn, *tensors) / small(fn, *tensors): run fn() on the side stream (after the main
    stream's work so far) if the mode sends that class there, else in place; join(): the main
    stream waits for every fork. Everything runs in place on CPU tensors or with mode 0."""

    def __init__(self, dev, mode=None):
        self.mode = MODE if mode is None else mode
        self.side = _side_stream(dev) if (self.mode and dev.type == "cuda") else None
        self.dev = dev
        self.keep = []

    def _fork(self, fn, tensors):
        self.side.wait_stream(torch.cuda.current_stream(self.dev))
        self.keep.extend(tensors)
        with torch.cuda.stream(self.side):
            return fn()

    def big(self, fn, *tensors):
        if self.side is None or self.mode != 1:
            return fn()
        return self._fork(fn, tensors)

    def small(self, fn, *tensors):
        if self.side is None:
            return fn()
        return self._fork(fn, tensors)

    def join(self):
        if self.side is not None:
            torch.cuda.current_stream(self.dev).wait_stream(self.side)
        self.keep.clear()
