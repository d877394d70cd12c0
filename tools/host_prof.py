"""Host-side (Python) cost of the eager config-2 step: cProfile over K eager steps, top functions by
own time, plus the wall time per step with and without a device sync per step.

  python tools/host_prof.py [K]
"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402
ge.add_pkg_path()
import torch  # noqa: E402


def main():
    import bench
    from engine.dp import DataParallelStep
    from engine.train import batch_to_device
    from train_utils.load_sources import load_sources
    from dataset import synthetic
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 10

    class Args:
        batch, points, parts, sources = 16, 2048, 4, 512
    cfg = bench.workload_cfg(Args)
    dev = torch.device("cuda:0")
    db, _ = load_sources(cfg, dev)
    step = DataParallelStep(cfg, db, dev)
    bs = [batch_to_device(synthetic.make_batch(16, 2048, db.num_sources, parts=4, seed=i), dev, db.num_sources)
          for i in range(4)]
    for i in range(3):
        step.step(bs[i % 4])
    torch.cuda.synchronize()
    # host issue time: launches queue up asynchronously; time the Python side only
    t0 = time.perf_counter()
    for i in range(K):
        step.step(bs[i % 4])
    t_issue = (time.perf_counter() - t0) / K
    torch.cuda.synchronize()
    t_all = (time.perf_counter() - t0) / K
    print(f"host issue {t_issue * 1e3:.2f} ms/step, wall {t_all * 1e3:.2f} ms/step")
    pr = cProfile.Profile()
    pr.enable()
    for i in range(K):
        step.step(bs[i % 4])
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(35)


if __name__ == "__main__":
    main()
