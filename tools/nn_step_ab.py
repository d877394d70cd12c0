"""A/B of the chamfer NN forward paths inside the config-2 step's loss families:
time compute_cm_loss (full + part families, fwd+bwd) and the whole train step with the
fused forward enabled / disabled (ured_hip.nn.FUSED).

  python tools/nn_step_ab.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402
ge.add_pkg_path()
import torch  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    import bench
    from engine.train import TrainStep, batch_to_device, get_part
    from train_utils.load_sources import load_sources
    from dataset import synthetic
    from loss.chamfer_loss import compute_cm_loss
    from ured_hip import nn as unn

    class Args:
        batch, points, parts, sources = 16, 2048, 4, 512
    cfg = bench.workload_cfg(Args)
    dev = torch.device("cuda:0")
    db, _ = load_sources(cfg, dev)
    ts = TrainStep(cfg, db, dev)
    batch = batch_to_device(synthetic.make_batch(16, 2048, db.num_sources, parts=4, seed=0), dev, db.num_sources)
    loss, T = ts.forward(batch)
    out = T["_out"].detach().requires_grad_(True)
    x = batch["x"]
    M = ts.models
    with torch.no_grad():
        tc, pp = M["target_encoder_full"].forward_pointmajor(x, M["embedding_layer"](batch["tgt_sem"]))
    tpf, _, re_in, mask, part_x, param_def = get_part(cfg, pp.view(16, 2048, -1), batch["labels"], x)

    def losses():
        a, b = compute_cm_loss(out, x, part_x, mask)
        (a + b).backward()
    res = {}
    for fused in (True, False, True, False):
        unn.FUSED = fused
        tag = "fused" if fused else "two_pass"
        res[tag + "_cm_loss_ms"] = round(timeit(losses), 4)
        res[tag + "_step_ms"] = round(timeit(lambda: ts.step(batch)), 4)
    unn.FUSED = True
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
