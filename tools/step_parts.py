"""GPU time of the config-2 step's parts in isolation (fwd + bwd each, CUDA events), to
attribute the step time: encoders, residual nets, DeformNet, losses, optimizer.

  python tools/step_parts.py
"""
import os
import sys
import json

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402
ge.add_pkg_path()
import torch  # noqa: E402


def timeit(fn, iters=10):
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
    from engine.train import TrainStep, batch_to_device
    from train_utils.load_sources import load_sources
    from dataset import synthetic
    from loss.chamfer_loss import compute_cm_loss
    from loss.basic_loss import residual_retrieval_loss
    from loss.contrast_loss import compute_contrast_loss_loss
    from dataset.dataset_utils import get_symmetric

    class Args:
        batch, points, parts, sources = 16, 2048, 4, 512
    cfg = bench.workload_cfg(Args)
    dev = torch.device("cuda:0")
    db, _ = load_sources(cfg, dev)
    ts = TrainStep(cfg, db, dev)
    batch = batch_to_device(synthetic.make_batch(16, 2048, db.num_sources, parts=4, seed=0), dev, db.num_sources)
    res = {}
    res["step"] = timeit(lambda: ts.step(batch))
    res["fwd_only"] = timeit(lambda: ts.forward(batch))
    M = ts.models
    B, P, C = 16, 16, cfg["source_latent_dim"]
    tcode = torch.randn(B, C, device=dev, requires_grad=True)
    codes = torch.randn(B, P, C, device=dev, requires_grad=True)

    def deform():
        out = M["param_decoder_full"](tcode, codes, None)
        out.sum().backward()
    res["deformnet_fwd_bwd"] = timeit(deform)
    res["deformnet_fwd"] = timeit(lambda: M["param_decoder_full"](tcode, codes, None))
    loss, T = ts.forward(batch)
    out = T["_out"].detach().requires_grad_(True)
    x = batch["x"]
    from engine.train import get_part
    with torch.no_grad():
        tc, pp = M["target_encoder_full"].forward_pointmajor(x, M["embedding_layer"](batch["tgt_sem"]))
    tpf, _, re_in, mask, part_x, param_def = get_part(cfg, pp.view(B, 2048, -1), batch["labels"], x)

    def losses():
        a, b = compute_cm_loss(out, x, part_x, mask)
        c, d = compute_cm_loss(get_symmetric(out), x, part_x, mask)
        e, f = residual_retrieval_loss(x, out.detach(), out[:, :2048].detach().clone().requires_grad_(True), mask)
        (30 * a + b + 30 * c + 3 * e + 0.03 * f).backward()
    res["chamfer_losses_fwd_bwd"] = timeit(losses)
    tpf2 = tpf.detach().requires_grad_(True)
    lab = torch.where(batch["src_labels"] >= 0, torch.ones_like(batch["src_labels"]), batch["src_labels"])
    res["contrast_fwd_bwd"] = timeit(lambda: compute_contrast_loss_loss(tpf2, codes, lab).backward())
    res["get_part"] = timeit(lambda: get_part(cfg, pp.view(B, 2048, -1), batch["labels"], x))
    ts.step(batch)
    res["clip_and_adam"] = timeit(ts.clip_and_step)
    uq = batch["src_unique"]
    from ured_hip.kernels import RowWeights
    rw = RowWeights(uq.w, 1024)
    pts = db.points[uq.uniq].unsqueeze(0)
    sem = M["embedding_layer"](db.sem[uq.uniq]).detach().unsqueeze(0)

    def src_enc():
        c, p = M["src_encoder_all"].forward_pointmajor(pts, sem, rw=rw)
        r = M["recon_decoder_src"].forward_split(p, c, code_first=True, group_rows=1024, rw=rw)
        (c.sum() + r.sum()).backward()
    res["src_encoder+recon_fwd_bwd"] = timeit(src_enc)
    tsem = M["embedding_layer"](batch["tgt_sem"]).detach()

    def tgt_enc():
        c, p = M["target_encoder_full"].forward_pointmajor(x, tsem)
        r = M["recon_decoder_full"].forward_split(p, c, group_rows=2048)
        r2 = M["re_residual_net_full"].forward_split(re_in.pp_sorted.detach(), re_in.part_mean.detach(),
                                                     gidx=re_in.gid, off=re_in.off)
        (c.sum() + r.sum() + r2.sum()).backward()
    res["tgt_encoder+2res_fwd_bwd"] = timeit(tgt_enc)
    print(json.dumps({k: round(v, 3) for k, v in res.items()}, indent=1))


if __name__ == "__main__":
    main()
