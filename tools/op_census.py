"""Census of the small torch ops one config-2 train step dispatches, attributed to the first
frame inside the package (forward) or to the autograd node being run (backward).

  python tools/op_census.py > out.txt
"""
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402
ge.add_pkg_path()
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

PKG = os.path.basename(ge.PKG_DIR)
SKIP = {"aten.view.default", "aten._unsafe_view.default", "aten.t.default", "aten.transpose.int",
        "aten.expand.default", "aten.as_strided.default", "aten.detach.default", "aten.permute.default",
        "aten.unsqueeze.default", "aten.squeeze.dim", "aten.select.int", "aten.slice.Tensor",
        "aten.alias.default", "aten.empty.memory_format", "aten.empty_strided.default", "aten.reshape.default",
        "aten._reshape_alias.default", "aten.split.Tensor", "aten.unbind.int", "aten.empty_like.default",
        "aten.lift_fresh.default", "aten.new_empty.default", "aten.new_empty_strided.default", "aten.is_same_size.default",
        "aten.squeeze.default", "aten.unsqueeze_.default", "aten.split_with_sizes.default", "aten.chunk.default",
        "aten.narrow.default", "aten.diagonal.default", "aten.movedim.int", "aten.flatten.using_ints",
        "aten.resize_.default", "aten.set_.source_Storage_storage_offset", "aten._to_copy.default"}


class Census(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.c = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func)
        if name not in SKIP:
            where = "backward/autograd"
            for fr in reversed(traceback.extract_stack()[:-1]):
                if "op_census" in fr.filename:
                    continue
                if PKG in fr.filename or "/tools/" in fr.filename or "/engine/" in fr.filename:
                    where = f"{os.path.relpath(fr.filename, ROOT)}:{fr.lineno} {fr.name}"
                    break
            self.c[(name, where)] += 1
        return func(*args, **(kwargs or {}))


def main():
    import bench
    from engine.dp import DataParallelStep
    from engine.train import batch_to_device
    from train_utils.load_sources import load_sources
    from dataset import synthetic

    class Args:
        batch, points, parts, sources = 16, 2048, 4, 512
    cfg = bench.workload_cfg(Args)
    dev = torch.device("cuda:0")
    db, _ = load_sources(cfg, dev)
    step = DataParallelStep(cfg, db, dev)
    b = batch_to_device(synthetic.make_batch(16, 2048, db.num_sources, parts=4, seed=0), dev, db.num_sources)
    for _ in range(2):
        step.step(b)
    torch.cuda.synchronize()
    m = Census()
    with m:
        step.step(b)
    torch.cuda.synchronize()
    tot = sum(m.c.values())
    print("total ops", tot)
    by_op = collections.Counter()
    for (op, _), n in m.c.items():
        by_op[op] += n
    for op, n in by_op.most_common(40):
        print(f"{n:5d} {op}")
    print()
    for (op, where), n in m.c.most_common(150):
        print(f"{n:4d} {op:45s} {where}")


if __name__ == "__main__":
    main()
