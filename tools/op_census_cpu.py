"""CPU dry run of tools/op_census.py: the torch ops one config-2 train step dispatches, with every
libured_hip.so entry point stubbed out (no GPU needed). Tensors are zero-filled instead of
uninitialised so that indices the stubbed kernels would have produced stay in range. Numbers are
meaningless; the op list is the step's (the HIP launches themselves are not torch ops).

  python tools/op_census_cpu.py [--batch 16 --points 2048] > out.txt
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import __graft_entry__ as ge  # noqa: E402
ge.add_pkg_path()
import torch  # noqa: E402

from ured_hip import _lib  # noqa: E402

_real_empty = torch.empty


def _zeros_empty(*a, **k):
    return torch.zeros(*a, **k)


def stub():
    _lib.call = lambda name, *a: None
    _lib.stream_of = lambda t: None
    _lib.current_stream = lambda: None
    _lib.require_device = lambda *t: None
    import ured_hip.mlp as mlp
    mlp._nbt = lambda bnm: bnm.num_batches_tracked
    import types
    torch.cuda.current_stream = lambda *a, **k: types.SimpleNamespace(cuda_stream=0)
    torch.empty = _zeros_empty
    torch.Tensor.record_stream = lambda self, s: None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--points", type=int, default=2048)
    ap.add_argument("--parts", type=int, default=4)
    ap.add_argument("--top", type=int, default=150)
    a = ap.parse_args()
    stub()
    import bench
    from op_census import Census
    from engine.train import TrainStep, batch_to_device
    from train_utils.load_sources import load_sources
    from dataset import synthetic

    class Args:
        batch, points, parts, sources = a.batch, a.points, a.parts, 512
    cfg = bench.workload_cfg(Args)
    cfg["device"] = "cpu"
    dev = torch.device("cpu")
    db, _ = load_sources(cfg, dev)
    step = TrainStep(cfg, db, dev)
    # the GPU path's choices (CPU tensors would pick the composed forms)
    step.loss_head = cfg.get("loss_head", True)
    import functools
    import engine.train as et
    from ured_hip import ops
    et.build_parts = functools.partial(ops.build_parts, composed=False)
    # the GPU step's optimizer (train_utils/optimizer_dm.py picks it for device parameters only)
    from ured_hip.optim import FlatAdam
    from engine.train import CLIPPED
    mods = [step.models[n] for n in CLIPPED]
    step.optimizer = FlatAdam([p for m in mods for p in m.parameters()], [list(m.parameters()) for m in mods],
                              lr=cfg["learning_rate"], weight_decay=cfg["weight_decay"])
    b =batch_to_device(synthetic.make_batch(a.batch, a.points, db.num_sources, parts=a.parts, seed=0), dev,
                        db.num_sources)
    step.step(b)
    class NodeCensus(Census):
        """Backward ops attributed to the autograd node being run, with the output shape."""

        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            node = torch._C._current_autograd_node()
            if node is None:
                return Census.__torch_dispatch__(self, func, types, args, kwargs)
            out = func(*args, **(kwargs or {}))
            name = str(func)
            from op_census import SKIP
            if name != "aten.zeros.default" and name not in SKIP and name != "aten.detach.default":
                shp = tuple(out.shape) if torch.is_tensor(out) else ""
                self.c[(name, f"bwd {node.name()} {shp}")] += 1
            return out

    m = NodeCensus()
    with m:
        step.step(b)
    tot = sum(m.c.values())
    print("total ops", tot)
    by_op = collections.Counter()
    for (op, _), n in m.c.items():
        by_op[op] += n
    for op, n in by_op.most_common(50):
        print(f"{n:5d} {op}")
    print()
    for (op, where), n in m.c.most_common(a.top):
        print(f"{n:4d} {op:45s} {where}")


if __name__ == "__main__":
    main()
