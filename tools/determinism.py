"""Run-to-run check of the HIP train step: the same forward + backward twice on one batch, every
parameter gradient compared bitwise (prints the ones that differ and by how much).

  python tools/determinism.py [--bs 8 --points 2048] [--poison 1e30]

--poison V: every float torch.empty/empty_like is filled with V before use (runs 1 and 2; run 0
uses plain torch.empty), so a kernel that reads memory nobody wrote shows up as a difference.
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

ge.add_pkg_path()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bs", type=int, default=8)
    ap.add_argument("--points", type=int, default=2048)
    ap.add_argument("--poison", type=float, default=None)
    a = ap.parse_args()
    real_empty, real_empty_like = torch.empty, torch.empty_like

    def poisoned(fn):
        def f(*args, **kw):
            t = fn(*args, **kw)
            if t.is_floating_point() and t.is_cuda:
                t.fill_(a.poison)
            return t
        return f
    from dataset import synthetic
    from engine.train import TrainStep, batch_to_device
    from train_utils.load_sources import SourceDB
    dev = torch.device("cuda:0")
    with open(os.path.join(ge.PKG_DIR, "config", "config_train_test.json")) as f:
        cfg = json.load(f)
    cfg.update(device="cuda", log_every=0, batch_size=a.bs)
    dbn = synthetic.make_source_db(512, seed=3)
    db = SourceDB(dbn["src_points"], dbn["src_mats"], dbn["src_default_param"], dbn["src_sem"], dev)
    torch.manual_seed(11)
    step = TrainStep(cfg, db, dev)
    batch = batch_to_device(synthetic.make_batch(a.bs, a.points, 512, parts=4, seed=5), dev, 512)
    # the first encoder layer's weight-gradient inputs and output, per run (ured_hip.mlp)
    import ured_hip.mlp as umlp
    real_lw = umlp._enc_layer_wgrad
    layer0 = []

    pre_sync = os.environ.get("DET_SYNC") == "1"

    def spy(spec, i, N, M, G, GR, x, sem, Ys, states, dYi, cs, W, dW):
        if i == 0:
            if pre_sync:
                torch.cuda.synchronize()
            pre = (x.clone(), dYi.clone())
        real_lw(spec, i, N, M, G, GR, x, sem, Ys, states, dYi, cs, W, dW)
        if i == 0:
            if not (torch.equal(pre[0], x) and torch.equal(pre[1], dYi)):
                print(f"layer-0 wgrad ({spec.mode}): inputs changed across the call")
            got = dW.clone()
            torch.cuda.synchronize()
            again = torch.empty_like(dW)           # the same weight gradient, recomputed in isolation
            real_lw(spec, i, N, M, G, GR, x, sem, Ys, states, dYi, cs, W, again)
            torch.cuda.synchronize()
            if not torch.equal(got, again):
                print(f"layer-0 wgrad ({spec.mode}): in-step result != isolated recompute, "
                      f"max |d| {(got - again).abs().max().item():.3e}")
            layer0.append((spec.mode, x.clone(), dYi.clone(), cs.clone(), got))
    umlp._enc_layer_wgrad = spy
    grads, losses = [], []
    for r in range(3):
        if a.poison is not None and r > 0:
            torch.empty, torch.empty_like = poisoned(real_empty), poisoned(real_empty_like)
        step.optimizer.zero_grad(set_to_none=True)
        loss, T = step.forward(batch, 1)
        loss.backward()
        losses.append(float(loss))
        grads.append({f"{m}.{k}": p.grad.detach().clone() for m in step.models
                      for k, p in step.models[m].named_parameters() if p.grad is not None})
    print("losses", losses)
    bad = 0
    for k in grads[0]:
        for r in (1, 2):
            if not torch.equal(grads[0][k], grads[r][k]):
                d = (grads[0][k] - grads[r][k]).abs().max().item()
                print(f"run {r} differs: {k} max |d| {d:.3e} (max |g| {grads[0][k].abs().max().item():.3e})")
                bad += 1
    per = len(layer0) // 3
    for j in range(per):
        for r in (1, 2):
            a0, a1 = layer0[j], layer0[r * per + j]
            diff = [nm for nm, u, v in zip(("x", "dY", "cs", "dW"), a0[1:], a1[1:]) if not torch.equal(u, v)]
            if diff:
                print(f"layer-0 wgrad call {j} ({a0[0]}) run {r}: differs in {diff}")
    print("deterministic" if bad == 0 else f"{bad} gradient tensors differ")


if __name__ == "__main__":
    main()
