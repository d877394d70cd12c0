"""§8(f)2: device pseudo-label selection (train_utils/pseudo_labels.py) vs the line-by-line
restatement of get_labels / mask_label / check_similarity (oracle/pseudo_label_ref.py).
Integer labels: bit-exact. The table logic is plain torch device ops, so the CPU suite
checks it on CPU tensors and the GPU suite on the MI355X."""
import numpy as np
import pytest
import torch

from oracle import pseudo_label_ref as ref


def _case(seed, T=200, NS=300, B=16, P=16):
    rng = np.random.Generator(np.random.PCG64(seed))
    cd_m = rng.uniform(0.0, 0.05, size=(T, NS))
    cd_m[rng.uniform(size=T) < 0.2] += 0.05                 # rows with nothing under alpha
    for t in range(0, T, 7):                                 # near-duplicate rows -> same choices
        cd_m[t + 1:t + 3] = cd_m[t] + rng.uniform(0, 1e-9, size=(min(t + 3, T) - t - 1, NS))
    part_sem = rng.integers(0, 6, size=T)
    sources_sem = rng.integers(0, 6, size=NS)
    pos = rng.uniform(size=NS)
    dist_src = np.abs(pos[:, None] - pos[None, :]) + rng.uniform(0, 1e-3, size=(NS, NS))
    dist_src = dist_src + dist_src.T
    np.fill_diagonal(dist_src, 0.0)
    rows = np.full((B, P), -1, np.int64)
    lists = []
    for b in range(B):
        k = int(rng.integers(1, P + 1))
        base = int(rng.integers(0, T - 3))
        r = rng.integers(0, T, size=k)
        r[: min(k, 3)] = np.arange(base, base + min(k, 3))  # a run of near-duplicate parts
        rows[b, :k] = r
        lists.append(r.tolist())
    return cd_m, part_sem, sources_sem, dist_src, rows, lists


def _check(dev, seed):
    from train_utils.pseudo_labels import PseudoLabelTable
    cd_m, part_sem, sources_sem, dist_src, rows, lists = _case(seed)
    tab = PseudoLabelTable(cd_m, part_sem, sources_sem, dist_src, alpha=2e-2, cl_k=40, device=dev)
    got = tab.labels(torch.from_numpy(rows).to(dev)).cpu().numpy()
    exp = ref.get_labels(lists, cd_m, part_sem, sources_sem, dist_src, 2e-2, 40, rows.shape[1])
    np.testing.assert_array_equal(got, exp)
    assert (exp == -1).sum() > (rows == -1).sum()            # some parts were masked
    return got


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_labels_cpu_match_reference(seed):
    _check("cpu", seed)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 3])
def test_labels_gpu_match_reference(dev, seed):
    _check(dev, seed)


@pytest.mark.gpu
def test_pickles_end_to_end(dev, tmp_path):
    """PairGenerator.cross (target parts x sources, calc_dcd on HIP) -> per-part pickles in the
    reference format -> PseudoLabelTable.from_pickles -> labels == the oracle reading the same
    pickles; the table built straight from cross() gives the same labels."""
    import pickle
    from dataset import synthetic
    from engine.generate_pair import PairGenerator, normalize_pts
    from train_utils.pseudo_labels import PseudoLabelTable
    NS, T = 96, 24
    src = np.stack([normalize_pts(p) for p in synthetic.make_source_db(NS, seed=3)["src_points"]])
    tgt = np.stack([normalize_pts(p) for p in synthetic.make_source_db(T, seed=4)["src_points"]])
    gen = PairGenerator(torch.from_numpy(src).to(dev))
    table = gen.cross(torch.from_numpy(tgt))                  # [3, T, NS]
    cd_m = table[2].double().cpu().numpy()
    names = [f"tgt{t:03d}_0" for t in range(T)]
    for t, n in enumerate(names):
        with open(tmp_path / (n + ".pickle"), "wb") as f:
            pickle.dump({"dcd_loss": table[0, t].double().cpu().numpy(), "cd_s": table[1, t].double().cpu().numpy(),
                         "cd_m": cd_m[t]}, f)
    rng = np.random.Generator(np.random.PCG64(0))
    part_sem, sources_sem = rng.integers(0, 3, size=T), rng.integers(0, 3, size=NS)
    d = gen.rows(range(NS))
    from engine.generate_pair import connect_matrix
    dist_src = connect_matrix(d, NS)[2]
    alpha = float(np.quantile(cd_m, 0.05))
    rows = np.full((4, 16), -1, np.int64)
    lists = [[0, 1, 2], [3, 4, 5, 6, 7, 8], list(range(9, 24)), [5, 5]]
    for b, l in enumerate(lists):
        rows[b, :len(l)] = l
    tab = PseudoLabelTable.from_pickles(str(tmp_path), names, part_sem, sources_sem, dist_src,
                                        alpha=alpha, cl_k=10, device=dev)
    got = tab.labels(torch.from_numpy(rows).to(dev)).cpu().numpy()
    exp = ref.get_labels(lists, cd_m, part_sem, sources_sem, dist_src, alpha, 10, 16)
    np.testing.assert_array_equal(got, exp)
    direct = PseudoLabelTable(table[2], part_sem, sources_sem, dist_src, alpha=alpha, cl_k=10)
    np.testing.assert_array_equal(direct.labels(torch.from_numpy(rows).to(dev)).cpu().numpy(), exp)
    # the cross table is calc_dcd(x = target, gt = source): the [t, s] pair of the dense path
    d1, d2, i1, i2 = __import__("ured_hip.nn", fromlist=["nn_dense"]).nn_dense(
        torch.from_numpy(src[5:6]).to(dev), torch.from_numpy(tgt[7:8]).to(dev))
    from ured_hip.nn import dcd
    np.testing.assert_array_equal(torch.stack(dcd(d1, i1, d2, i2)).squeeze(1).cpu().numpy(),
                                  table[:, 7, 5].cpu().numpy())


def _golden():
    import os
    from conftest import GOLDEN
    return np.load(os.path.join(GOLDEN, "pseudo_labels.npz"))


def test_oracle_matches_reference_golden():
    """oracle/pseudo_label_ref.py vs the reference's own get_labels / mask_label /
    check_similarity / read_pickle_topk (tests/golden/make_golden.py golden_pseudo_labels:
    lifted from dataset/dataset_utils.py:1043-1143, pickle reads from an in-memory table)."""
    g = _golden()
    rows = g["part_rows"]
    lists = [[int(r) for r in row if r >= 0] for row in rows]
    exp = ref.get_labels(lists, g["cd_m"], g["part_sem"], g["sources_sem"], g["dist_src"], float(g["alpha"]),
                         int(g["cl_k"]), rows.shape[1])
    np.testing.assert_array_equal(exp, g["source_labels"])


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_table_matches_reference_golden(device, request):
    """PseudoLabelTable (the device path that replaces the per-iteration pickle reads) vs the
    reference's get_labels on the same table: integer labels bit-exact."""
    from train_utils.pseudo_labels import PseudoLabelTable
    if device == "cuda":
        device = request.getfixturevalue("dev")
    g = _golden()
    tab = PseudoLabelTable(g["cd_m"], g["part_sem"], g["sources_sem"], g["dist_src"], alpha=float(g["alpha"]),
                           cl_k=int(g["cl_k"]), device=device)
    got = tab.labels(torch.from_numpy(g["part_rows"]).to(device)).cpu().numpy()
    np.testing.assert_array_equal(got, g["source_labels"])


def test_part_bounds_cover_every_part():
    """PartBounds (the loss head's NN launch bounds) are >= the parts per target and the points
    per part of every target, rounded up (to a multiple of 4 parts; to a power of two >= 256
    points), from the host labels alone."""
    from ured_hip.ops import PartBounds
    rng = np.random.default_rng(5)
    for trial in range(20):
        B, N = int(rng.integers(1, 5)), int(rng.integers(1, 3000))
        k = rng.integers(1, 17, size=B)
        lab = np.stack([rng.integers(0, kk, size=N) for kk in k])
        pb = PartBounds(lab)
        for row in lab:
            _, c = np.unique(row, return_counts=True)
            assert c.shape[0] <= pb.k and c.max() <= pb.count
        assert pb.k % 4 == 0 and pb.count >= 256 and pb.count & (pb.count - 1) == 0
        assert pb.k - max(np.unique(r).shape[0] for r in lab) < 4
        most = max(np.unique(r, return_counts=True)[1].max() for r in lab)
        assert pb.count == 256 or pb.count < 2 * most
