"""§8(f)3 inference-side pieces: NDCG@40 retrieval score (cal_retrieval_score,
dataset/dataset_utils.py:1165-1176) against sklearn.metrics.ndcg_score itself (present in this
image: the reference's own dependency), and the batched mesh deformation against the
reference's get_shape_numpy (dataset_utils.py:601-621) applied per part."""
import numpy as np
import pytest
import torch


def _scores(seed, Q=12, L=300, ties=False):
    rng = np.random.Generator(np.random.PCG64(seed))
    cd = rng.uniform(0, 0.004, size=(Q, L))
    score = rng.uniform(-1, 1, size=(Q, L))
    if ties:
        score = np.round(score * 8) / 8                  # many exact ties in the ranking
    return cd, score


@pytest.mark.parametrize("ties", [False, True])
@pytest.mark.parametrize("aligned", [False, True])
def test_ndcg_matches_sklearn(ties, aligned):
    from sklearn.metrics import ndcg_score as sk_ndcg
    from dataset.dataset_utils import cal_retrieval_score
    cd, score = _scores(3 + ties, ties=ties)
    got = cal_retrieval_score(torch.from_numpy(score), torch.from_numpy(cd), k=40, aligned=aligned).numpy()
    for q in range(cd.shape[0]):
        d = cd[q] if aligned else np.sort(cd[q])        # read_pickle_topk returns sorted distances
        rel = np.exp(-np.asarray(d) ** 2 / (2.0 * 0.001 ** 2))
        exp = sk_ndcg([rel.tolist()], [score[q].tolist()], k=40)
        assert abs(got[q] - exp) <= 1e-12 * max(1.0, abs(exp)), (q, got[q], exp)


def test_ndcg_all_irrelevant_is_zero():
    from dataset.dataset_utils import ndcg_score
    z = ndcg_score(torch.zeros(2, 50, dtype=torch.float64), torch.rand(2, 50, dtype=torch.float64), 40)
    assert torch.equal(z, torch.zeros(2, dtype=torch.float64))


def _mesh_case(dev):
    from dataset import synthetic
    db = synthetic.make_source_db(20, seed=5)
    m = synthetic.make_source_meshes(db, seed=6, vmin=5, vmax=40)
    rng = np.random.Generator(np.random.PCG64(7))
    src = rng.integers(-1, 20, size=(3, 4))
    src = np.where(src < 0, src + 20, src)
    params = rng.standard_normal((3, 4, 6)).astype(np.float32)
    pdef = rng.uniform(0, 1, (3, 4, 6)).astype(np.float32)
    return m, src, params, pdef


def _check_mesh(dev):
    from dataset.dataset_utils import deform_vertices, get_shape_numpy
    m, src, params, pdef = _mesh_case(dev)
    v, off = deform_vertices(torch.from_numpy(m["vmats"]).to(dev), torch.from_numpy(m["voff"]).to(dev),
                             torch.from_numpy(src).to(dev), torch.from_numpy(params).to(dev),
                             torch.from_numpy(pdef).to(dev), 0.1)
    v, off = v.cpu().numpy(), off.cpu().numpy()
    for b in range(3):
        for i in range(4):
            s = src[b, i]
            A = m["vmats"][m["voff"][s]:m["voff"][s + 1]]
            exp = get_shape_numpy(A, params[b, i].reshape(1, 6, 1), pdef[b, i].reshape(6, 1), 0.1)
            slot = b * 4 + i
            np.testing.assert_allclose(v[off[slot]:off[slot + 1]], exp.reshape(-1, 3), rtol=1e-6, atol=1e-6)
            # A = [I | diag(q)]: the deformed vertex is t + q*s exactly as the mesh generator built it
            assert off[slot + 1] - off[slot] == (m["voff"][s + 1] - m["voff"][s]) // 3


def test_deform_vertices_cpu():
    _check_mesh("cpu")


@pytest.mark.gpu
def test_deform_vertices_gpu(dev):
    _check_mesh(dev)


@pytest.mark.gpu
def test_ndcg_gpu_matches_cpu(dev):
    from dataset.dataset_utils import cal_retrieval_score
    cd, score = _scores(9, Q=64, L=5232, ties=True)
    a = cal_retrieval_score(torch.from_numpy(score).to(dev), torch.from_numpy(cd).to(dev)).cpu()
    b = cal_retrieval_score(torch.from_numpy(score), torch.from_numpy(cd))
    torch.testing.assert_close(a, b, rtol=1e-12, atol=1e-12)
