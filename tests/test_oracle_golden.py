"""Pin the oracle (CPU restatement) against golden vectors generated from the
reference itself (tests/golden/make_golden.py). CPU only."""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import nn_ref, ured_ref

sys.path.insert(0, GOLDEN)
from sketch import STEP_CASES, grad_sketch  # noqa: E402  (tests/golden/sketch.py)

CFG = {"source_latent_dim": 64, "target_latent_dim": 64, "sem_latent_dim": 16, "MAX_NUM_PARTS": 16,
       "alpha": 0.1, "use_chamfer_loss": 30.0, "use_chamfer_part_loss": 1.0, "use_symmetry_loss": 30.0,
       "use_contrast_loss": 0.5, "use_param_loss": 0.0, "init_p_m_loss": -1, "use_residuals_reg": 3.0,
       "use_recon": 30.0}
SEED = 7


def _g(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def test_nn_oracle_vs_distchamfer():
    """chamfer_python.distChamfer is the reference's own oracle (unit_test.py:14-35):
    MSE < 1e-8 and exact index equality on random data."""
    g = _g("nn_distchamfer.npz")
    for case in ("u4x100x200", "u3x257x129", "u2x1x5", "u1x2048x2048"):
        d1, d2, i1, i2 = nn_ref.nn_fwd(g[case + "/p1"], g[case + "/p2"])
        assert np.mean((d1 - g[case + "/d1"]) ** 2) + np.mean((d2 - g[case + "/d2"]) ** 2) < 1e-8
        assert np.abs(d1 - g[case + "/d1"]).max() < 1e-6 and np.abs(d2 - g[case + "/d2"]).max() < 1e-6
        np.testing.assert_array_equal(i1, g[case + "/i1"])
        np.testing.assert_array_equal(i2, g[case + "/i2"])


def test_dist_chamfer_restatement_vs_reference():
    """oracle.nn_ref.dist_chamfer (the CPU baseline's chamfer, bench.py) restates the reference's
    chamfer_python.distChamfer: bit-exact on the reference-generated golden vectors."""
    for case in ("u4x100x200", "u3x257x129", "u2x1x5", "u1x2048x2048", "grid"):
        g = _g("nn_distchamfer.npz")
        d1, d2, i1, i2 = nn_ref.dist_chamfer(torch.from_numpy(g[case + "/p1"]), torch.from_numpy(g[case + "/p2"]))
        np.testing.assert_array_equal(d1.numpy(), g[case + "/d1"])
        np.testing.assert_array_equal(d2.numpy(), g[case + "/d2"])
        np.testing.assert_array_equal(i1.numpy(), g[case + "/i1"])
        np.testing.assert_array_equal(i2.numpy(), g[case + "/i2"])


def _direct_sq(q, r):
    q = q.astype(np.float32); r = r.astype(np.float32)
    dx = r[None, :, 0] - q[:, None, 0]; dy = r[None, :, 1] - q[:, None, 1]; dz = r[None, :, 2] - q[:, None, 2]
    inner = (dy.astype(np.float64) * dy + (dx * dx).astype(np.float64)).astype(np.float32)  # fmaf(dy,dy,dx*dx)
    return (dz.astype(np.float64) * dz + inner.astype(np.float64)).astype(np.float32)      # fmaf(dz,dz,inner)


def test_nn_oracle_ties_lowest_index():
    """Grid refs with exact fp32 ties: the reference keeps the first minimum (strict '<', chamfer3D.cu:36-69)."""
    g = _g("nn_distchamfer.npz")
    q, r = g["grid/p1"][0], g["grid/p2"][0]
    d, i = nn_ref.nn_dir(q, r)
    D = _direct_sq(q, r)
    assert np.abs(d - g["grid/d1"][0]).max() < 1e-6
    for j in range(q.shape[0]):
        assert D[j, i[j]] == d[j]
        assert i[j] == np.flatnonzero(D[j] == D[j].min())[0]
    assert (np.sum(D == D.min(axis=1, keepdims=True), axis=1) > 1).sum() >= 300  # the tie cases exist


def _req(P):
    for k, v in P.items():
        if v.dtype.is_floating_point and "running" not in k:
            v.requires_grad_(True)


def _params():
    return ured_ref.make_params(CFG, seed=SEED)


def test_target_encoder_golden():
    g = _g("modules.npz")
    P = _params()["target_encoder_full"]
    _req(P)
    x = torch.tensor(g["tgt/x"], requires_grad=True)
    s = torch.tensor(g["tgt/sem"], requires_grad=True)
    code, pp = ured_ref.target_encoder(P, x, s, False)
    np.testing.assert_allclose(code.detach().numpy(), g["tgt/code"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(pp.detach().numpy(), g["tgt/pp"], rtol=1e-4, atol=1e-5)
    ((code * torch.tensor(g["tgt/w1"])).sum() + (pp * torch.tensor(g["tgt/w2"])).sum()).backward()
    np.testing.assert_allclose(x.grad.numpy(), g["tgt/gx"], rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(s.grad.numpy(), g["tgt/gsem"], rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(P["fuse_sem.0.weight"].grad[:32].numpy(), g["tgt/g_fuse_w"], rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(P["mlp1.0.weight"].grad.numpy(), g["tgt/g_mlp10_w"], rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(P["per_point_out.3.weight"].grad.numpy(), g["tgt/g_ppo3_w"], rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(P["fc.weight"].grad.numpy(), g["tgt/g_fc_w"], rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(P["fuse_sem.1.running_mean"].detach().numpy(), g["tgt/rm_fuse"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(P["fuse_sem.1.running_var"].detach().numpy(), g["tgt/rv_fuse"], rtol=1e-4, atol=1e-6)
    with torch.no_grad():
        c_e, pp_e = ured_ref.target_encoder(P, x, s, False, training=False)
    np.testing.assert_allclose(c_e.numpy(), g["tgt_eval/code"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(pp_e.numpy(), g["tgt_eval/pp"], rtol=1e-4, atol=1e-5)


def test_source_encoder_golden():
    g = _g("modules.npz")
    P = _params()["src_encoder_all"]
    code, pp = ured_ref.target_encoder(P, torch.tensor(g["src/x"]), torch.tensor(g["src/sem"]), True)
    np.testing.assert_allclose(code.detach().numpy(), g["src/code"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(pp.detach().numpy(), g["src/pp"], rtol=1e-4, atol=1e-5)


def test_residual_net_golden():
    g = _g("modules.npz")
    P = _params()["recon_decoder_full"]
    _req(P)
    f = torch.tensor(g["res/in"], requires_grad=True)
    r = ured_ref.residual_net(P, f)
    np.testing.assert_allclose(r.detach().numpy(), g["res/out"], rtol=1e-4, atol=1e-5)
    (r * torch.tensor(g["res/w"])).sum().backward()
    np.testing.assert_allclose(f.grad.numpy(), g["res/gin"], rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(P["residual_net.0.weight"].grad.numpy(), g["res/g_w0"], rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(P["residual_net.9.weight"].grad.numpy(), g["res/g_w9"], rtol=1e-3, atol=1e-5)


def test_deform_net_golden():
    g = _g("modules.npz")
    P = _params()["param_decoder_full"]
    _req(P)
    tf = torch.tensor(g["dn/tf"], requires_grad=True)
    spf = torch.tensor(g["dn/spf"], requires_grad=True)
    prm = ured_ref.deform_net(P, tf, spf)
    np.testing.assert_allclose(prm.detach().numpy(), g["dn/params"], rtol=1e-4, atol=1e-5)
    (prm * torch.tensor(g["dn/w"])).sum().backward()
    np.testing.assert_allclose(tf.grad.numpy(), g["dn/gtf"], rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(spf.grad.numpy(), g["dn/gspf"], rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(P["param_decoder.0.weight"].grad.numpy(), g["dn/g_dec0_w"], rtol=1e-3, atol=1e-5)


def test_small_losses_golden():
    g = _g("modules.npz")
    a, b, m = torch.tensor(g["cons/a"]), torch.tensor(g["cons/b"]), torch.tensor(g["cons/mask"])
    np.testing.assert_allclose(ured_ref.pc_consistency(a[:, 0], b[:, 0]).numpy(), g["cons/plain"], rtol=1e-6)
    np.testing.assert_allclose(ured_ref.pc_consistency_weighted(a, b, m).numpy(), g["cons/weighted"], rtol=1e-6)
    loss = ured_ref.contrast_loss(torch.tensor(g["con/t"]), torch.tensor(g["con/s"]), torch.tensor(g["con/l"]))
    np.testing.assert_allclose(loss.numpy(), g["con/loss"], rtol=1e-6)


def synthetic_step_batch(parts=(3, 2), dtype=torch.float32):
    from dataset import synthetic
    db = synthetic.make_source_db(24, seed=3)
    bt = synthetic.make_batch(2, 128, 24, max_parts=16, parts=list(parts), seed=4)
    batch = {"src_points": torch.from_numpy(db["src_points"]).to(dtype), "src_mats": torch.from_numpy(db["src_mats"]).to(dtype),
             "src_sem": torch.from_numpy(db["src_sem"]), "src_index": torch.from_numpy(bt["src_index"]),
             "tgt_sem": torch.from_numpy(bt["tgt_sem"]), "x": torch.from_numpy(bt["x"]).to(dtype),
             "labels": torch.from_numpy(bt["labels"]).to(dtype), "src_labels": torch.from_numpy(bt["src_labels"])}
    return batch


_ENC_BN_FED = ("mlp1.0", "mlp1.3", "mlp2.0", "mlp2.3", "mlp2.6", "fuse_sem.0", "per_point_out.0")
BN_FED = {"src_encoder_all": _ENC_BN_FED, "target_encoder_full": _ENC_BN_FED}   # Conv -> BN (train)


def _sketch_dev(got, ref):
    """max |got - ref| / max(|ref|) of one stored part (elementwise, relative to the part's scale)."""
    return float(np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-30))


@pytest.mark.parametrize("fname", sorted(STEP_CASES))
def test_train_step_golden(fname):
    """The whole engine/train.py:192-338 step composed from the reference's own functions and
    modules, in float64 (tests/golden/make_golden.py golden_step), vs the oracle in float64:
    every loss term within 1e-6 relative, the deformed shape and DeformNet params within 1e-6
    of their scale, and EVERY parameter gradient elementwise — whole tensors up to 16 k elements,
    larger ones through row sums, column sums, 2048 sampled elements and 16 Gaussian projections
    (tests/golden/sketch.py) — within 1e-5 of the part's largest magnitude. (Both sides take their
    chamfer costs in fp32: the reference's distChamfer casts its float64 result, the oracle's C
    NN computes the fp32 contract; the rest is float64.) The conv biases feeding a training-mode
    BN and the attention key biases have an exactly-zero true gradient and are checked against
    a noise floor."""
    g = _g(fname)
    over, parts = STEP_CASES[fname]
    P = _params()
    for mod in P.values():
        for k in list(mod):
            if mod[k].dtype.is_floating_point:
                mod[k] = mod[k].double()
                if "running" not in k:
                    mod[k].requires_grad_(True)
    batch = synthetic_step_batch(parts, torch.float64)
    cfg = dict(dict(CFG, batch_size=2, complementme=False), **over)
    loss, T = ured_ref.train_forward(P, batch, cfg)
    np.testing.assert_allclose(T["_out"].detach().numpy(), g["out"], rtol=0, atol=1e-6 * np.abs(g["out"]).max())
    np.testing.assert_allclose(T["_params"].detach().numpy(), g["params_full"], rtol=0,
                               atol=1e-6 * np.abs(g["params_full"]).max())
    terms = [k[5:] for k in g.files if k.startswith("loss/")]
    assert ("param_loss" in terms) == (cfg.get("use_param_loss", 0) > 0)
    assert set(terms) == {k for k in T if not k.startswith("_")}
    worst = {}
    for k in terms:
        ref = float(g["loss/" + k])
        worst[k] = abs(float(T[k].detach()) - ref) / abs(ref)
        assert worst[k] <= 1e-6, f"{k}: {float(T[k].detach())} vs {ref}"
    print(f"\n{fname}: max loss-term rel dev {max(worst.values()):.2e}")
    loss.backward()
    nchecked, gdev = 0, 0.0
    names = {key.split("/", 1)[1] for key in g.files if key.startswith("gnorm/")}
    for mod in ured_ref.TRAINED_MODULES:        # every gradient the reference produced, and no other
        for k, v in P[mod].items():
            if torch.is_tensor(v) and v.requires_grad:
                assert (v.grad is not None) == (f"{mod}/{k}" in names), f"{mod}/{k}"
    for name in sorted(names):
        mod, k = name.split("/", 1)
        got = P[mod][k].grad
        sk = grad_sketch(name, got)
        if k.endswith(".bias") and (k[:-5] in BN_FED.get(mod, ()) or k.endswith("in_proj_k.bias")):
            # exactly-zero true gradients: a conv bias feeding a training-mode BN (the batch mean
            # removes it) and the attention key bias (q.b_k is the same for every key of a query:
            # softmax removes it) — rounding noise on both sides
            wn = float(g[f"gnorm/{mod}/{k[:-5]}.weight"])
            assert got.norm().item() <= 1e-6 * wn + 1e-10 and float(g["gnorm/" + name]) <= 1e-6 * wn + 1e-10, name
            continue
        for part, v in sk.items():
            ref = g[f"g/{name}/{part}"]
            if part == "idx":
                np.testing.assert_array_equal(v, ref)
                continue
            d = _sketch_dev(v, ref)
            gdev = max(gdev, d)
            assert d <= 1e-5, f"{name} [{part}]: max dev {d:.2e} of the part's scale"
        nchecked += 1
    print(f"{fname}: {nchecked} gradient tensors, max elementwise dev {gdev:.2e}")
    assert nchecked >= 145


def test_dcd_oracle_vs_reference_golden():
    """oracle.dcd_ref.calc_dcd vs the reference's calc_dcd (model_utils.py:13-51) run on the
    reference's float64 distChamfer (tests/golden/make_golden.py golden_dcd)."""
    from oracle import dcd_ref
    g = _g("dcd.npz")
    for name in ("r3x300x200", "r2x1024x1024", "r4x64x512"):
        x, gt = g[name + "/x"], g[name + "/gt"]
        for nr in (0, 1):
            loss, cd_p, cd_t = dcd_ref.calc_dcd(x, gt, non_reg=bool(nr))
            tag = f"{name}/nr{nr}"
            np.testing.assert_allclose(loss, g[tag + "/loss"], rtol=0, atol=2e-6)
            np.testing.assert_allclose(cd_p, g[tag + "/cd_p"], rtol=0, atol=2e-6)
            np.testing.assert_allclose(cd_t, g[tag + "/cd_t"], rtol=0, atol=2e-6)
        loss, _, _ = dcd_ref.calc_dcd(x, gt, alpha=200, n_lambda=2)
        np.testing.assert_allclose(loss, g[name + "/a200l2/loss"], rtol=0, atol=2e-6)


def test_pair_rows_connect_matrix():
    """get_src_pair rows + sources_connect composition (symmetric, diagonal doubled)."""
    from oracle import dcd_ref
    pts = np.random.Generator(np.random.PCG64(3)).random((5, 64, 3), dtype=np.float32)
    rows = dcd_ref.pair_rows(pts)
    assert [len(rows[i][0]) for i in range(5)] == [5, 4, 3, 2, 1]
    m = dcd_ref.connect_matrix(rows, 5)
    np.testing.assert_array_equal(m, m.transpose(0, 2, 1))
    d, _, _ = dcd_ref.calc_dcd(pts[3:4], pts[1:2])
    assert m[0, 1, 3] == np.float64(d[0])
    assert m[2, 2, 2] == 0.0 and abs(m[0, 2, 2] - 2e-6) < 1e-7   # self pair: dcd = 1 - 1/(1+1e-6)


def test_shard_rows_balanced_and_complete():
    import sys
    from conftest import PKG_DIR
    sys.path.insert(0, PKG_DIR)
    from engine.generate_pair import shard_rows
    for n in (1, 2, 7, 100, 513):
        for world in (1, 2, 3, 8):
            shards = [shard_rows(n, r, world) for r in range(world)]
            assert sorted(sum(shards, [])) == list(range(n))
            loads = [sum(n - i for i in s) for s in shards]
            if n >= 8 * world:
                assert max(loads) - min(loads) <= n + 1, (n, world, loads)   # at most one zig-zag pair
