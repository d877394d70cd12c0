"""Retrieval + deformation inference (engine/test.py, vis.py semantics) vs the oracle.

Retrieval indices must match exactly except where the oracle's top-2 cosine gap is below
1e-5 (a near tie that fp32 summation order may flip; such slots are counted and reported)."""
import numpy as np
import pytest
import torch

from oracle import ured_ref

pytestmark = pytest.mark.gpu

CFG = {"source_latent_dim": 64, "target_latent_dim": 64, "sem_latent_dim": 16, "MAX_NUM_PARTS": 16,
       "alpha": 0.1, "device": "cuda", "optimizer": "adam", "learning_rate": 1e-3, "weight_decay": 5e-4,
       "lr_stepsize": 3, "lr_decay": 0.5, "momentum": 0.9}


def test_inference_matches_oracle(dev):
    from dataset import synthetic
    from train_utils.load_sources import SourceDB
    from engine.train import get_models, batch_to_device
    from engine.test import infer
    ns = 600
    dbn = synthetic.make_source_db(ns, seed=11)
    bt = synthetic.make_batch(3, 256, ns, parts=[4, 2, 7], seed=12)
    db = SourceDB(dbn["src_points"], dbn["src_mats"], dbn["src_default_param"], dbn["src_sem"], dev)
    models, _, _ = get_models(CFG, dev)
    P = ured_ref.make_params(CFG, seed=5)
    for name, sd in P.items():
        sd = {k: (v + 0.05 if "running_var" in k else v) for k, v in sd.items()}   # non-trivial eval stats
        models[name].load_state_dict(sd, strict=True)
        P[name] = sd
    r = infer(models, db, batch_to_device(bt, dev), CFG)
    ob = {"src_points": torch.from_numpy(dbn["src_points"]), "src_mats": torch.from_numpy(dbn["src_mats"]),
          "src_sem": torch.from_numpy(dbn["src_sem"]), "x": torch.from_numpy(bt["x"]),
          "labels": torch.from_numpy(bt["labels"]).float(), "tgt_sem": torch.from_numpy(bt["tgt_sem"])}
    R = ured_ref.infer(P, ob, CFG)
    got, ref = r["retrieved"].cpu(), R["retrieved"]
    near = R["sim_top2_gap"] < 1e-5
    mism = (got != ref) & ~near
    assert int(mism.sum()) == 0, f"{int(mism.sum())} retrieval mismatches outside near-ties"
    assert int(((got != ref) & near).sum()) <= 2
    same = (got == ref).all(dim=1)
    cd, rcd = r["cd"].cpu(), R["cd"]
    np.testing.assert_allclose(cd[same].numpy(), rcd[same].numpy(), rtol=1e-4)
    np.testing.assert_allclose(r["params"].cpu()[same].numpy(), R["params"][same].numpy(), rtol=1e-3, atol=1e-5)


def test_inference_scores_and_meshes(dev):
    """vis.py's per-batch extras: residual score max_pts sum|r| (vis.py:221-231), NDCG@40 per
    target part (cal_retrieval_score, vs sklearn in tests/test_retrieval_metrics.py), and the
    retrieved meshes deformed with the target-part boxes (get_shape_numpy per part)."""
    from sklearn.metrics import ndcg_score as sk_ndcg
    from dataset import synthetic
    from dataset.dataset_utils import get_shape_numpy
    from train_utils.load_sources import SourceDB
    from engine.train import get_models, batch_to_device, get_part
    from engine.test import encode_sources, infer
    import torch.nn.functional as F
    ns = 300
    dbn = synthetic.make_source_db(ns, seed=21)
    mesh = synthetic.make_source_meshes(dbn, seed=22, vmin=10, vmax=60)
    bt = synthetic.make_batch(2, 256, ns, parts=[3, 5], seed=23)
    db = SourceDB(dbn["src_points"], dbn["src_mats"], dbn["src_default_param"], dbn["src_sem"], dev)
    models, _, _ = get_models(CFG, dev)
    b = batch_to_device(bt, dev)
    rng = np.random.Generator(np.random.PCG64(24))
    rel = torch.from_numpy(rng.uniform(0, 0.004, size=(2, 16, ns))).to(dev)
    meshes = {"vmats": torch.from_numpy(mesh["vmats"]).to(dev), "voff": torch.from_numpy(mesh["voff"]).to(dev)}
    codes = encode_sources(models, db)
    r = infer(models, db, b, CFG, codes, relevance=rel, meshes=meshes)
    # NDCG: the same similarity rows scored by sklearn
    with torch.no_grad():
        tcode, pp = models["target_encoder_full"].forward_pointmajor(b["x"], models["embedding_layer"](b["tgt_sem"]))
        part_f, _, _, mask, _, param_def = get_part(CFG, pp.view(2, 256, -1), b["labels"], b["x"])
        sim = (F.normalize(part_f, dim=-1, p=2) @ codes.t()).double().cpu().numpy()
    nd = r["ndcg"].cpu().numpy()
    for bb, k in enumerate((3, 5)):
        for i in range(16):
            if i >= k:
                assert np.isnan(nd[bb, i])
                continue
            true = np.exp(-np.sort(rel[bb, i].cpu().numpy()) ** 2 / (2.0 * 0.001 ** 2))
            assert abs(nd[bb, i] - sk_ndcg([true.tolist()], [sim[bb, i].tolist()], k=40)) < 1e-9
    assert r["re_score"].shape == (2,) and bool(torch.isfinite(r["re_score"]).all())
    # meshes
    v, off = r["vertices"].cpu().numpy(), r["vertex_off"].cpu().numpy()
    idx = r["retrieved"].cpu().numpy()
    idx = np.where(idx < 0, idx + ns, idx)
    params, pdef = r["params"].cpu().numpy(), param_def.cpu().numpy()
    for bb in range(2):
        for i in range(16):
            s = idx[bb, i]
            A = mesh["vmats"][mesh["voff"][s]:mesh["voff"][s + 1]]
            exp = get_shape_numpy(A, params[bb, i].reshape(1, 6, 1), pdef[bb, i].reshape(6, 1), 0.1).reshape(-1, 3)
            np.testing.assert_allclose(v[off[bb * 16 + i]:off[bb * 16 + i + 1]], exp, rtol=1e-5, atol=1e-6)


def test_graphed_inference_matches_eager(dev):
    """GraphedInfer (one HIP graph per batch shape) replays bit-identically to infer() for new
    batches of the captured shape."""
    from dataset import synthetic
    from train_utils.load_sources import SourceDB
    from engine.train import get_models, batch_to_device
    from engine.test import encode_sources, infer, GraphedInfer
    ns = 400
    dbn = synthetic.make_source_db(ns, seed=31)
    db = SourceDB(dbn["src_points"], dbn["src_mats"], dbn["src_default_param"], dbn["src_sem"], dev)
    models, _, _ = get_models(CFG, dev)
    codes = encode_sources(models, db)
    gi = GraphedInfer(models, db, CFG, codes)
    batches = [batch_to_device(synthetic.make_batch(3, 256, ns, parts=[4, 2, 7], seed=40 + i), dev)
               for i in range(3)]
    for i, b in enumerate(batches):
        got = gi(b)                               # first call: eager + capture; then replays
        ref = infer(models, db, b, CFG, codes)
        for k in ("retrieved", "params", "out", "cd", "re_score", "sim_top2_gap"):
            assert torch.equal(got[k], ref[k]), (i, k)
    assert len(gi.graphs) == 1
