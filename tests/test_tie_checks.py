"""The parity tests' tie rules (oracle/ured_ref.py max_pool, check_nn_choice), on CPU: another
implementation's discrete choice is accepted only within the bound its own values imply."""
import pytest
import torch

from oracle import ured_ref as R


def _gpu(hg):
    return lambda idx: hg.double().gather(2, idx.unsqueeze(-1)).squeeze(-1)


def test_max_pool_accepts_choice_within_fp32_deviation():
    h = torch.tensor([[[1.0, 3.0, 3.0 + 1e-7, 0.5]]], dtype=torch.float64)
    hg = torch.tensor([[[1.0, 3.0 + 2e-7, 3.0, 0.5]]], dtype=torch.float32)   # the other side's values
    rec = {}
    out = R.max_pool(h, torch.tensor([[1]]), rec, _gpu(hg))
    assert float(out) == 3.0 and rec["overridden"] == 1 and rec["near_ties"] == 1
    assert 0 < rec["max_gap_over_bound"] <= 1


def test_max_pool_rejects_wrong_winner():
    h = torch.tensor([[[1.0, 3.0, 3.01, 0.5]]], dtype=torch.float64)
    hg = h.float()
    with pytest.raises(AssertionError, match="not a near-tie"):
        R.max_pool(h, torch.tensor([[1]]), {}, _gpu(hg))


def test_max_pool_counts_exact_ties():
    h = torch.zeros(1, 2, 5, dtype=torch.float64)           # all-zero ReLU channels
    rec = {}
    R.max_pool(h, torch.tensor([[3, 1]]), rec, _gpu(h.float()))
    assert rec["exact_ties"] == 2 and rec["near_ties"] == 0 and rec["max_gap"] == 0.0


def test_nn_choice_bound():
    R.NN_TIE_STATS.clear()
    q = torch.tensor([[[0.0, 0.0, 0.0]]], dtype=torch.float64)
    c = torch.tensor([[[1.0, 0.0, 0.0], [1.0 + 1e-6, 0.0, 0.0]]], dtype=torch.float64)
    own, given = torch.tensor([[0]]), torch.tensor([[1]])
    R.check_nn_choice(q, c, given, own, torch.tensor([[1e-6]]), 0, "t")      # within 2 x the deviation
    assert R.NN_TIE_STATS["t"]["near_ties"] == 1
    with pytest.raises(AssertionError, match="not a near-tie"):
        R.check_nn_choice(q, c, given, own, torch.tensor([[1e-8]]), 0, "t")


def test_max_pool_rejects_wide_deviation():
    # the other side's value at its winner is far off: the bound built from it would accept the
    # wrong winner, so the deviation itself is rejected
    h = torch.tensor([[[1.0, 3.0, 3.01, 0.5]]], dtype=torch.float64)
    hg = torch.tensor([[[1.0, 3.5, 3.01, 0.5]]], dtype=torch.float32)
    with pytest.raises(AssertionError, match="its values are wrong"):
        R.max_pool(h, torch.tensor([[1]]), {}, _gpu(hg))


def test_nn_choice_rejects_wide_copy_deviation():
    q = torch.tensor([[[0.0, 0.0, 0.0]]], dtype=torch.float64)
    c = torch.tensor([[[1.0, 0.0, 0.0], [1.1, 0.0, 0.0]]], dtype=torch.float64)
    own, given = torch.tensor([[0]]), torch.tensor([[1]])
    with pytest.raises(AssertionError, match="its points are wrong"):
        R.check_nn_choice(q, c, given, own, torch.tensor([[0.2]]), 0, "t")
