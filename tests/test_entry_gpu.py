"""The drop-in entry points on the GPU: engine/train.py main() with the reference's pseudo-label
selection wired in (PseudoLabelLoader: target-part x source calc_dcd table + sources_connect,
labels bit-exact vs the line-by-line get_labels restatement, itself pinned to the reference by
tests/golden/pseudo_labels.npz), checkpoints in the reference format, and engine/test.py main()
loading them through the vis-style config schema."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import PKG_DIR
from oracle import pseudo_label_ref as ref

pytestmark = pytest.mark.gpu


def _cfg(tmp_path, **over):
    with open(os.path.join(PKG_DIR, "config", "config_train_test.json")) as f:
        cfg = json.load(f)
    cfg.update(source_latent_dim=64, target_latent_dim=64, part_latent_dim=64, sem_latent_dim=16, batch_size=2,
               num_points=256, num_source=48, num_targets=6, parts=3, epochs=2, save_epoch=1, log_every=1,
               log_path=str(tmp_path / "ws"), device="cuda", cl_k=8)
    cfg.update(over)
    os.makedirs(cfg["log_path"], exist_ok=True)
    return cfg


def test_pseudo_label_loader_matches_get_labels(dev, tmp_path):
    from engine.train import PseudoLabelLoader
    from train_utils.load_sources import load_sources
    cfg = _cfg(tmp_path, filter_threshold=1.0)
    db, dist_src = load_sources(cfg, dev)
    assert dist_src.shape == (48, 48) and np.allclose(dist_src, dist_src.T)   # the cd_m plane
    assert (dist_src > 0).mean() > 0.9
    ld = PseudoLabelLoader(cfg, db, dev, dist_src, seed=3)
    rows = ld.part_rows
    lists = [[int(r) for r in row if r >= 0] for row in rows]
    exp = ref.get_labels(lists, ld.table.cd_m.cpu().numpy(), ld.table.part_sem.cpu().numpy(), db.sem.cpu().numpy(),
                         dist_src, cfg["filter_threshold"], cfg["cl_k"], cfg["MAX_NUM_PARTS"])
    got = ld.table.labels(torch.from_numpy(rows).to(dev)).cpu().numpy()
    np.testing.assert_array_equal(got, exp)
    assert (exp[:, :3] >= 0).any()
    n = 0
    for b in ld:                        # each batch's labels drawn on the device when it is drawn
        assert b["x"].shape == (2, 256, 3)
        np.testing.assert_array_equal(b["src_labels"].cpu().numpy(), exp[ld.last_sel])
        n += 1
    assert n == 3
    # targets assembled from source parts: most parts are labelled with their own source
    own = ld.targets["src_true"]
    k = own.shape[1]
    assert (exp[:, :k][own >= 0] == own[own >= 0]).mean() > 0.5


def test_train_then_test_main(dev, tmp_path):
    from engine import test as etest
    from engine import train as etrain
    cfg = _cfg(tmp_path)
    trainer = etrain.main(cfg)
    ck = os.path.join(cfg["log_path"], "checkpoint_0001.pth")
    assert os.path.exists(ck) and os.path.exists(os.path.join(cfg["log_path"], "checkpoint_0000.pth"))
    sd = torch.load(ck, map_location="cpu", weights_only=True)
    assert set(sd) == {"target_encoder_full", "param_decoder_full", "re_residual_net_full", "recon_decoder_full",
                       "src_encoder_all", "recon_decoder_src", "embedding_layer"}
    for name, m in trainer.models.items():
        for k, v in m.state_dict().items():
            assert torch.equal(sd[name][k], v.cpu()), (name, k)
    with open(os.path.join(PKG_DIR, "config", "config_vis_test.json")) as f:
        vcfg = json.load(f)
    vcfg.update(source_latent_dim=64, target_latent_dim=64, part_latent_dim=64, sem_latent_dim=16, batch_size=2,
                num_points=256, num_source=48, iters_per_epoch=1, dm_model_path=ck, re_model_path=ck,
                log_path=cfg["log_path"])
    etest.main(vcfg)
    with pytest.raises(FileNotFoundError):
        etest.main(dict(vcfg, dm_model_path=str(tmp_path / "missing.pth")))
