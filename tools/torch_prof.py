"""torch.profiler view of one config-2 train step: which torch ops launch the small kernels.

  python tools/torch_prof.py [--steps 2] > out.txt
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402
ge.add_pkg_path()
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--stacks", action="store_true", help="group the small ops by Python call stack")
    ap.add_argument("--shapes", action="store_true", help="list the torch GEMMs by input shape")
    a = ap.parse_args()
    import bench
    from engine.dp import DataParallelStep
    from engine.train import batch_to_device
    from train_utils.load_sources import load_sources
    from dataset import synthetic

    class Args:
        batch, points, parts, sources = 16, 2048, 4, 512
    cfg = bench.workload_cfg(Args)
    dev = torch.device("cuda:0")
    torch.backends.cuda.preferred_blas_library("cublas")   # rocBLAS, as bench.py's default --blas
    db, _ = load_sources(cfg, dev)
    step = DataParallelStep(cfg, db, dev)
    batches = [batch_to_device(synthetic.make_batch(16, 2048, db.num_sources, parts=4, seed=i), dev, db.num_sources)
               for i in range(2)]
    for i in range(3):
        step.step(batches[i % 2])
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=a.shapes,
                 with_stack=a.stacks) as prof:
        for i in range(a.steps):
            step.step(batches[i % 2])
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_device_time_total", row_limit=70, max_name_column_width=60))
    print(prof.key_averages(group_by_stack_n=0).table(sort_by="count", row_limit=40, max_name_column_width=60))
    if a.shapes:
        rows = [e for e in prof.key_averages(group_by_input_shape=True)
                if e.key in ("aten::mm", "aten::addmm", "aten::bmm", "aten::matmul", "aten::linear")]
        rows.sort(key=lambda e: -e.device_time_total)
        for e in rows[:40]:
            print(f"{e.key:12s} n={e.count:4d} dev_us={e.device_time_total:9.1f} {e.input_shapes}")
    if a.stacks:
        want = ("aten::add", "aten::add_", "aten::fill_", "aten::zero_", "aten::sum", "aten::copy_",
                "aten::mul", "aten::cat", "aten::mm", "aten::addmm", "aten::bmm", "aten::div")
        rows = [e for e in prof.key_averages(group_by_stack_n=6) if e.key in want]
        rows.sort(key=lambda e: -e.device_time_total)
        for e in rows[:60]:
            print(f"{e.key:14s} n={e.count:4d} dev_us={e.device_time_total:9.1f}")
            for fr in e.stack[:6]:
                print("      ", fr)


if __name__ == "__main__":
    main()
