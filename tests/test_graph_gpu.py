"""The HIP-graph step (engine/graph.py) replays exactly the eager step: same losses and the
same parameters, bitwise, over several steps with changing batches."""
import pytest
import torch

from test_dp_gpu import CFG

pytestmark = pytest.mark.gpu


def _make(dev, cfg):
    from dataset import synthetic
    from engine.dp import DataParallelStep
    from oracle import ured_ref
    from train_utils.load_sources import SourceDB
    dbn = synthetic.make_source_db(24, seed=3)
    db = SourceDB(dbn["src_points"], dbn["src_mats"], dbn["src_default_param"], dbn["src_sem"], dev)
    step = DataParallelStep(cfg, db, dev)
    for name, sd in ured_ref.make_params(cfg, seed=7).items():
        step.models[name].load_state_dict(sd, strict=True)
    return step


def test_graph_replay_equals_eager(dev):
    from dataset import synthetic
    from engine.graph import GraphedStep
    from engine.train import batch_to_device
    cfg = dict(CFG, cuda_graph=True)
    batches = [batch_to_device(synthetic.make_batch(2, 128, 24, parts=[3, 2], seed=50 + i), dev) for i in range(4)]
    a, b = _make(dev, cfg), _make(dev, cfg)
    g = GraphedStep(a, batches[0], warmup=3)          # 3 eager steps on batch 0, then capture
    for _ in range(3):
        b.step(batches[0])
    for i in range(1, 4):
        la = g.step(batches[i])["all_loss"].clone()
        lb = b.step(batches[i])["all_loss"]
        assert torch.equal(la, lb), (i, la.item(), lb.item())
    for name in ("src_encoder_all", "param_decoder_full", "re_residual_net_full"):
        for (k, pa), (_, pb) in zip(a.models[name].state_dict().items(), b.models[name].state_dict().items()):
            assert torch.equal(pa, pb), (name, k)
