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


def test_graph_replay_unique_sources_equals_eager(dev):
    """Unique-source batches padded to buckets: one captured graph per padded count (two keys
    here), replays bitwise-equal to eager steps on the same batches; padding groups (weight 0)
    change nothing."""
    from dataset import synthetic
    from engine.graph import GraphedStep
    from engine.train import batch_to_device
    cfg = dict(CFG, cuda_graph=True)
    parts = [[3, 2], [5, 4], [3, 2], [5, 4], [2, 2]]
    batches = [batch_to_device(synthetic.make_batch(2, 128, 24, parts=p, seed=70 + i), dev, 24, bucket=4)
               for i, p in enumerate(parts)]
    keys = {(b["src_unique"].U, b["part_bounds"].key()) for b in batches}   # GraphedStep.key's batch part
    assert len(keys) >= 2
    a, b = _make(dev, cfg), _make(dev, cfg)
    g = GraphedStep(a)
    for i in range(2):
        b.step(batches[0])
        g.step(batches[0])
    for rnd in range(2):
        for i, bt in enumerate(batches):
            la = g.step(bt)["all_loss"].clone()
            lb = b.step(bt)["all_loss"]
            assert torch.equal(la, lb), (rnd, i, la.item(), lb.item())
    assert len(g.graphs) == len(keys)
    for name in ("src_encoder_all", "recon_decoder_src", "param_decoder_full"):
        for (k, pa), (_, pb) in zip(a.models[name].state_dict().items(), b.models[name].state_dict().items()):
            assert torch.equal(pa, pb), (name, k)


def test_padded_unique_rows_match_unpadded(dev):
    """Zero-weight padding groups leave losses and gradients unchanged (up to summation order)."""
    from dataset import synthetic
    from engine.train import batch_to_device
    bt = synthetic.make_batch(2, 128, 24, parts=[3, 2], seed=90)
    p = batch_to_device(bt, dev, 24, bucket=16)
    u = batch_to_device(bt, dev, 24)
    assert p["src_unique"].U > u["src_unique"].U
    a, b = _make(dev, CFG), _make(dev, CFG)
    la, Ta = a.forward(p)
    lb, Tb = b.forward(u)
    assert abs(la.item() - lb.item()) <= 1e-6 * abs(lb.item())
    la.backward()
    lb.backward()
    for (k, pa), (_, pb) in zip(a.models["src_encoder_all"].named_parameters(),
                                b.models["src_encoder_all"].named_parameters()):
        if pa.grad is None:
            continue
        assert (pa.grad - pb.grad).norm() <= 1e-4 * pb.grad.norm() + 1e-6, k


def test_graph_replay_across_residual_gate(dev):
    """init_p_m_loss = 0: the residual loss switches on at epoch 1 (engine/train.py:306-316). The
    graphs captured at epoch 0 must not be replayed afterwards (the gate is part of the key; the
    set of parameters with a gradient changes, so everything is re-captured): graph steps equal
    eager steps bitwise across the flip, and the residual net trains only from epoch 1."""
    from dataset import synthetic
    from engine.graph import GraphedStep
    from engine.train import batch_to_device
    cfg = dict(CFG, cuda_graph=True, init_p_m_loss=0)
    batches = [batch_to_device(synthetic.make_batch(2, 128, 24, parts=[3, 2], seed=60 + i), dev) for i in range(3)]
    a, b = _make(dev, cfg), _make(dev, cfg)
    g = GraphedStep(a)
    r0 = {k: p.detach().clone() for k, p in a.models["re_residual_net_full"].named_parameters()}
    for ep, i in ((0, 0), (0, 1), (0, 2), (1, 0), (1, 1), (1, 2), (1, 0)):
        Ta = g.step(batches[i], epoch=ep)
        Tb = b.step(batches[i], epoch=ep)
        assert torch.equal(Ta["all_loss"], Tb["all_loss"]), (ep, i)
        assert ("re_reg_loss_full" in Ta) == (ep >= 1)
        if ep == 0:
            for k, p in a.models["re_residual_net_full"].named_parameters():
                assert torch.equal(p.detach(), r0[k]), k
    assert not torch.equal(a.models["re_residual_net_full"].residual_net[0].weight.detach(),
                           r0["residual_net.0.weight"])
    for name in a.models:
        for (k, pa), (_, pb) in zip(a.models[name].state_dict().items(), b.models[name].state_dict().items()):
            assert torch.equal(pa, pb), (name, k)


@pytest.mark.parametrize("opt", ["adam", "sgd"])
def test_graph_replay_follows_scheduler_with_torch_optimizers(dev, opt):
    """torch's Adam / SGD (cfg flat_adam: false, or optimizer sgd) bake the float learning rate
    into the captured update graph: GraphedStep re-captures that graph when StepLR changes the
    lr, so replayed steps across a scheduler step equal eager steps bitwise (FlatAdam reads its
    lr from a device scalar instead)."""
    from dataset import synthetic
    from engine.graph import GraphedStep
    from engine.train import batch_to_device
    cfg = dict(CFG, cuda_graph=True, flat_adam=False, optimizer=opt, momentum=0.9, lr_stepsize=1, lr_decay=0.5)
    batches = [batch_to_device(synthetic.make_batch(2, 128, 24, parts=[3, 2], seed=90 + i), dev) for i in range(3)]
    a, b = _make(dev, cfg), _make(dev, cfg)
    assert not hasattr(a.optimizer, "sync_lr")
    g = GraphedStep(a)
    for ep in range(3):
        for bt in batches:
            la = g.step(bt)["all_loss"].clone()
            lb = b.step(bt)["all_loss"]
            assert torch.equal(la, lb), (ep, la.item(), lb.item())
        g.scheduler.step()
        b.scheduler.step()
    assert g.update_captures >= 3                      # one per learning rate
    for name in a.models:
        for (k, pa), (_, pb) in zip(a.models[name].state_dict().items(), b.models[name].state_dict().items()):
            assert torch.equal(pa, pb), (name, k)
