"""The reference's config keys that change the loop (CPU): "mode" (engine/train.py:160-165,174:
batch size 2 and the dataset order when mode != "train") and the sources_connect plane key."""
import numpy as np
import pytest


def _cfg(**kw):
    cfg = {"batch_size": 16, "MAX_NUM_PARTS": 16, "num_points": 64, "parts": 3, "iters_per_epoch": 2}
    cfg.update(kw)
    return cfg


@pytest.mark.parametrize("mode,bs,shuffle", [("train", 16, True), ("test", 2, False), ("val", 2, False)])
def test_mode_sets_batch_size_and_order(mode, bs, shuffle):
    from engine.train import SyntheticLoader, loader_batching
    cfg = _cfg(mode=mode)
    assert loader_batching(cfg) == (bs, shuffle)
    batches = list(SyntheticLoader(cfg, 24, "cpu"))
    assert len(batches) == 2 and all(b["x"].shape[0] == bs for b in batches)


def test_mode_defaults_to_train():
    from engine.train import loader_batching
    assert loader_batching(_cfg()) == (16, True)


def test_mode_is_a_reference_key():
    from engine.config import EXTRA, REFERENCE_READS
    assert "mode" in REFERENCE_READS and "mode" not in EXTRA


def test_connectivity_plane_key():
    from train_utils.load_sources import connectivity_matrix
    n = 5
    stack = np.stack([np.full((n, n), float(i)) for i in range(3)])
    assert connectivity_matrix(stack, n)[0, 0] == 2.0                 # default: cd_m
    assert connectivity_matrix(stack, n, plane=0)[0, 0] == 0.0
    assert connectivity_matrix(np.eye(n), n, plane=0)[0, 0] == 1.0    # a 2-D matrix is taken as is
    with pytest.raises(ValueError):
        connectivity_matrix(stack, n, plane=3)
    with pytest.raises(ValueError):
        connectivity_matrix(np.zeros((4, 4)), n)
