"""CPU restatement of the U-RED training step — TEST INFRASTRUCTURE ONLY.

This is the parity checker for the HIP path (and the cpu_baseline leg of
bench.py). It is written functionally over plain state_dict-keyed parameter
dicts, following (reference root = the U-RED repo):

  TargetEncoder.forward          network/simple_encoder.py:88-107
  re_residual_net.forward        network/deformation_net.py:96-107 (+ FeedForwardNet_norm,
                                 attention_graph/attention_utils.py:62-86: Conv -> ReLU -> BN)
  DeformNet_MatchingNet.forward  network/deformation_net.py:74-93
  GraphAttentionNet & co.        attention_graph/attention_gnn.py:8-98, attention.py:8-19
  get_part                       engine/train.py:103-136 (+ compute_aabbox dataset/dataset_utils.py:77-85)
  get_shape / get_symmetric      dataset/dataset_utils.py:691-726, :1194-1196
  compute_cm_loss                loss/chamfer_loss.py:5-30
  residual_retrieval_loss        loss/basic_loss.py:249-265
  consistency losses             loss/basic_consistency_loss.py:4-22
  contrast loss                  loss/contrast_loss.py:61-102
  regularization_param           loss/regularization_loss.py:49-53 (cfg["use_param_loss"] > 0)
  complementme z-flip            engine/train.py:192-194 (cfg["complementme"])
  loss assembly / optimiser      engine/train.py:196-345, train_utils/optimizer_dm.py:68-104

Pinned against reference-generated golden vectors (tests/golden/make_golden.py).
Shape_Measure.ChamferLoss is absent from the reference tree (unpinned); it is
taken to return squared NN distances, as the in-tree chamfer_3DDist does.
"""
import math
from collections import OrderedDict

import numpy as np
import torch
import torch.nn.functional as F

from . import nn_ref

BN_EPS = 1e-5
BN_MOMENTUM = 0.1

# ----------------------------------------------------------------------------
# architecture description -> state_dict key/shape lists (same keys as the reference)
# ----------------------------------------------------------------------------


def _conv(prefix, cin, cout, k=True):
    return [(prefix + ".weight", (cout, cin, 1) if k else (cout, cin), "w", cin),
            (prefix + ".bias", (cout,), "b", cin)]


def _bn(prefix, c):
    return [(prefix + ".weight", (c,), "gamma", c), (prefix + ".bias", (c,), "beta", c),
            (prefix + ".running_mean", (c,), "rm", c), (prefix + ".running_var", (c,), "rv", c),
            (prefix + ".num_batches_tracked", (), "nbt", c)]


def _stn_keys(prefix, cin):
    k = []
    k += _conv(prefix + ".mlp1.0", cin, 64) + _bn(prefix + ".mlp1.1", 64)
    k += _conv(prefix + ".mlp1.3", 64, 128) + _bn(prefix + ".mlp1.4", 128)
    k += _conv(prefix + ".mlp1.6", 128, 1024) + _bn(prefix + ".mlp1.7", 1024)
    k += _conv(prefix + ".mlp2.0", 1024, 512, False) + _bn(prefix + ".mlp2.1", 512)
    k += _conv(prefix + ".mlp2.3", 512, 256, False) + _bn(prefix + ".mlp2.4", 256)
    k += _conv(prefix + ".mlp2.6", 256, cin * cin, False)
    return k


def target_encoder_keys(emb, sem, cin=3):
    k = _stn_keys("stn1", cin) + _stn_keys("stn2", 64)
    k += _conv("mlp1.0", cin, 64) + _bn("mlp1.1", 64) + _conv("mlp1.3", 64, 64) + _bn("mlp1.4", 64)
    k += _conv("mlp2.0", 64, 64) + _bn("mlp2.1", 64) + _conv("mlp2.3", 64, 128) + _bn("mlp2.4", 128)
    k += _conv("mlp2.6", 128, 1024) + _bn("mlp2.7", 1024)
    k += _conv("fuse_sem.0", 1024 + sem, 1024) + _bn("fuse_sem.1", 1024)
    k += _conv("per_point_out.0", 1024, emb) + _bn("per_point_out.1", emb) + _conv("per_point_out.3", emb, emb)
    k += _conv("fc", 1024, emb, False)
    return k


def ffn_norm_keys(prefix, dims, use_bn):
    k, i = [], 0
    for a, b in zip(dims[:-2], dims[1:-1]):
        k += _conv(f"{prefix}.{i}", a, b)
        if use_bn:
            k += _bn(f"{prefix}.{i + 2}", b)
            i += 3
        else:
            i += 2
    k += _conv(f"{prefix}.{i}", dims[-2], dims[-1])
    return k


def residual_net_keys(cin):
    return ffn_norm_keys("residual_net", [cin, 256, 256, 32, 3], True)


def deform_net_keys(c, num_stages=2, part_latent_dim=256):
    k = ffn_norm_keys("part_encoding", [part_latent_dim, 128, c], False)
    k += ffn_norm_keys("param_decoder", [3 * c, 256, 6], False)
    for L in range(2 * num_stages):
        p = f"graph_attention_net.layers.{L}.module"
        for nm in ("in_proj_q", "in_proj_k", "in_proj_v", "out_proj"):
            k += _conv(f"{p}.mha.{nm}", c, c)
        k += ffn_norm_keys(f"{p}.fc", [2 * c, 2 * c, c], True)
    return k


def model_keys(cfg):
    C, S = cfg["source_latent_dim"], cfg["sem_latent_dim"]
    Ct = cfg["target_latent_dim"]
    return OrderedDict([
        ("target_encoder_full", target_encoder_keys(Ct, S)),
        ("param_decoder_full", deform_net_keys(C)),
        ("re_residual_net_full", residual_net_keys(2 * Ct)),
        ("recon_decoder_full", residual_net_keys(2 * Ct)),
        ("src_encoder_all", target_encoder_keys(C, S)),
        ("recon_decoder_src", residual_net_keys(2 * C)),
        ("embedding_layer", [("weight", (42, S), "emb", S)]),
    ])


def make_params(cfg, seed=0, bn_jitter=0.1):
    """Deterministic parameters for every reference state_dict key.

    Weights/biases ~ U(-1/sqrt(fan_in), 1/sqrt(fan_in)) (torch's default bound),
    BN gamma = 1 + jitter*U(-1,1), beta = jitter*U(-1,1), running stats (0, 1),
    embedding ~ N(0,1). Each tensor has its own PCG64 stream keyed by its name.
    """
    out = OrderedDict()
    for mod, keys in model_keys(cfg).items():
        sd = OrderedDict()
        for name, shape, kind, fan in keys:
            h = int.from_bytes(f"{mod}.{name}".encode(), "little") % (2 ** 63)
            rng = np.random.Generator(np.random.PCG64([seed, h % (2 ** 32), h >> 32]))
            if kind in ("w", "b"):
                bound = 1.0 / math.sqrt(fan)
                v = rng.uniform(-bound, bound, size=shape)
            elif kind == "gamma":
                v = 1.0 + bn_jitter * rng.uniform(-1, 1, size=shape)
            elif kind == "beta":
                v = bn_jitter * rng.uniform(-1, 1, size=shape)
            elif kind == "rm":
                v = np.zeros(shape)
            elif kind == "rv":
                v = np.ones(shape)
            elif kind == "nbt":
                sd[name] = torch.tensor(0, dtype=torch.int64)
                continue
            elif kind == "emb":
                v = rng.standard_normal(size=shape)
            else:
                raise ValueError(kind)
            sd[name] = torch.tensor(np.asarray(v, dtype=np.float32).reshape(shape))
        out[mod] = sd
    return out


# ----------------------------------------------------------------------------
# layers (x is channel-first [B, C, N] like the reference's Conv1d inputs)
# ----------------------------------------------------------------------------


def conv(x, P, name):
    return F.conv1d(x, P[name + ".weight"], P[name + ".bias"])


def bn(x, P, name, training=True):
    return F.batch_norm(x, P[name + ".running_mean"], P[name + ".running_var"],
                        P[name + ".weight"], P[name + ".bias"], training, BN_MOMENTUM, BN_EPS)


U32 = 2.0 ** -24          # fp32 unit roundoff
DEV_TOL = 1e-4            # largest accepted deviation of the other implementation's pooled activations, of the layer scale (measured: <= 1.9e-6, profiles/r5b_gpu_tests.log)
NN_DEV_TOL = 1e-3         # ... and of its copy of a point set (the deformed shape: 1e-4 absolute in the step tests)


def max_pool(h, pool_idx=None, record=None, gpu_h=None):
    """max_pool1d over points (simple_encoder.py:105): h [G, C, N] -> [G, C].

    pool_idx (optional, [G, C] point index per channel): the winners another implementation (the
    HIP step) chose; they are taken instead of this function's argmax after a check derived from
    that implementation's own values, gpu_h(pidx [G, C]) -> its activation at those points: its
    winner w is a maximum of ITS values (ties to the lowest point), so with m this function's
    argmax, h[m] - h[w] = (h[m] - h_gpu[m]) + (h_gpu[m] - h_gpu[w]) + (h_gpu[w] - h[w]) <=
    |h[m] - h_gpu[m]| + |h_gpu[w] - h[w]|: the gap between the two choices may not exceed the two
    points' fp32 deviations (+ a few ulp of the channel's values). Anything wider is a wrong
    winner and raises. record gets "argmax" and the tie statistics: "overridden", "exact_ties"
    (gap exactly 0: e.g. channels whose ReLU output is 0 at both points), "near_ties",
    "max_gap" (absolute), "max_gap_rel" (over the channel's max |h|), "max_gap_over_bound"."""
    mx, am = h.max(dim=2)
    if record is not None:
        record["argmax"] = am.detach()
    if pool_idx is None:
        return mx
    if gpu_h is None:
        raise ValueError("max_pool: pool_idx needs gpu_h (the other implementation's values) for the tie check")
    idx = pool_idx.to(am.device).long()
    chosen = h.gather(2, idx.unsqueeze(-1)).squeeze(-1)
    gap = (mx - chosen).detach()
    hd = h.detach()
    dev_w = (gpu_h(idx).to(hd.dtype) - chosen.detach()).abs()
    dev_m = (gpu_h(am).to(hd.dtype) - mx.detach()).abs()
    # the deviations the bound is built from must themselves be small: a wrong GPU
    # activation may not widen the tolerance enough to accept a wrong winner
    # activation, relative to the layer's scale in that group (fp32 error follows the magnitudes
    # the channel was computed from, not the channel's own, possibly near-cancelled, maximum)
    g_scale = hd.abs().amax(dim=(1, 2)).unsqueeze(1) + 1e-30
    dev_rel = (torch.maximum(dev_w, dev_m) / g_scale)
    if bool((dev_rel > DEV_TOL).any()):
        g, c = [int(v) for v in (dev_rel > DEV_TOL).nonzero()[0]]
        raise AssertionError(f"max-pool tie check: the other implementation's activation at group {g} channel {c} "
                             f"deviates {float(dev_rel[g, c]):.3e} of the layer scale (> {DEV_TOL:.0e}): "
                             "its values are wrong, not its tie choice")
    bound = dev_w + dev_m + 4 * U32 * (mx.detach().abs() + chosen.detach().abs())
    over = idx != am
    bad = gap > bound
    if bool(bad.any()):
        g, c = [int(v) for v in bad.nonzero()[0]]
        raise AssertionError(f"max-pool winner {int(idx[g, c])} of group {g} channel {c} is {float(gap[g, c]):.3e} "
                             f"below the max ({float(mx[g, c]):.6e}), beyond the fp32 deviation bound "
                             f"{float(bound[g, c]):.3e}: not a near-tie")
    if record is not None:
        scale = hd.abs().amax(dim=2) + 1e-30
        g_o = gap[over]
        record.update(overridden=int(over.sum()), exact_ties=int((g_o == 0).sum()), near_ties=int((g_o > 0).sum()),
                      max_gap=float(g_o.max()) if g_o.numel() else 0.0,
                      max_gap_rel=float((gap / scale)[over].max()) if g_o.numel() else 0.0,
                      max_gap_over_bound=float((gap / (bound + 1e-300))[over].max()) if g_o.numel() else 0.0,
                      max_dev_rel=float(dev_rel.max()))
    return chosen


def target_encoder(P, x, sem_f, is_src, training=True, pool_idx=None, record=None, gpu_h=None):
    """network/simple_encoder.py:88-107. x: [B,N,3] (tgt) or [B,P,N,3] (src). pool_idx /
    record / gpu_h: see max_pool."""
    if is_src:
        B, Pn, N, _ = x.shape
        x = x.reshape(B * Pn, N, 3)
    N = x.shape[-2]
    h = x.transpose(2, 1)
    h = F.relu(bn(conv(h, P, "mlp1.0"), P, "mlp1.1", training))
    h = F.relu(bn(conv(h, P, "mlp1.3"), P, "mlp1.4", training))
    h = F.relu(bn(conv(h, P, "mlp2.0"), P, "mlp2.1", training))
    h = F.relu(bn(conv(h, P, "mlp2.3"), P, "mlp2.4", training))
    h = F.relu(bn(conv(h, P, "mlp2.6"), P, "mlp2.7", training))
    if is_src:
        s = sem_f.reshape(B * Pn, -1, 1).expand(-1, -1, N)
    else:
        s = sem_f.transpose(2, 1)
    h = torch.cat([h, s], dim=1)
    h = F.relu(bn(conv(h, P, "fuse_sem.0"), P, "fuse_sem.1", training))
    pp = F.relu(bn(conv(h, P, "per_point_out.0"), P, "per_point_out.1", training))
    pp = conv(pp, P, "per_point_out.3")
    g = max_pool(h, pool_idx, record, gpu_h)
    g = F.linear(g, P["fc.weight"], P["fc.bias"])
    return g, pp


def ffn_norm(h, P, prefix, nlayers, use_bn, training=True):
    i = 0
    for _ in range(nlayers - 1):
        h = F.relu(conv(h, P, f"{prefix}.{i}"))
        if use_bn:
            h = bn(h, P, f"{prefix}.{i + 2}", training)
            i += 3
        else:
            i += 2
    return conv(h, P, f"{prefix}.{i}")


def residual_net(P, feat, training=True):
    """network/deformation_net.py:102-107: feat [B,N,in] -> [B,N,3]."""
    return ffn_norm(feat.permute(0, 2, 1), P, "residual_net", 4, True, training).permute(0, 2, 1)


def _mha(P, p, q, kv, heads):
    B, C, _ = q.shape
    d = C // heads
    Q = conv(q, P, p + ".in_proj_q").view(B, heads, d, -1)
    K = conv(kv, P, p + ".in_proj_k").view(B, heads, d, -1)
    V = conv(kv, P, p + ".in_proj_v").view(B, heads, d, -1)
    att = torch.matmul(Q.transpose(2, 3), K) * d ** -0.5
    att = att.softmax(dim=-1)
    o = torch.matmul(att, V.transpose(2, 3)).transpose(2, 3).reshape(B, C, -1)
    return conv(o, P, p + ".out_proj")


def _prop(P, p, dq, dkv, heads, training):
    msg = _mha(P, p + ".mha", dq, dkv, heads)
    return dq + ffn_norm(torch.cat([dq, msg], dim=1), P, p + ".fc", 2, True, training)


def deform_net(P, target_f, src_part_f, num_stages=2, heads=4, training=True):
    """network/deformation_net.py:74-93 -> params [B, P, 6]."""
    B = target_f.shape[0]
    Pn = src_part_f.shape[1]
    parts = src_part_f.reshape(B, Pn, -1).permute(0, 2, 1)
    glob = torch.stack([parts.mean(dim=-1), target_f], dim=-1)
    for L in range(2 * num_stages):
        p = f"graph_attention_net.layers.{L}.module"
        if L % 2 == 0:   # self attention, shared module for both node sets
            glob, parts = _prop(P, p, glob, glob, heads, training), _prop(P, p, parts, parts, heads, training)
        else:            # cross attention
            g2 = _prop(P, p, glob, parts, heads, training)
            parts = _prop(P, p, parts, g2, heads, training)
            glob = g2
    gr = torch.cat([glob[:, :, 0], glob[:, :, 1]], dim=1).unsqueeze(-1).expand(-1, -1, Pn)
    full = torch.cat([gr, parts], dim=1)
    return ffn_norm(full, P, "param_decoder", 2, False, training).permute(0, 2, 1).contiguous()


# ----------------------------------------------------------------------------
# geometry glue
# ----------------------------------------------------------------------------


def get_part(per_point, labels, x, max_parts):
    """engine/train.py:103-136. per_point [B,N,C], labels [B,N] (float or int), x [B,N,3]."""
    B = per_point.shape[0]
    C = per_point.shape[-1]
    target_part_f, re_in, part_x = [], [], []
    mask = torch.zeros(B, max_parts)
    param_def = torch.zeros(B, max_parts, 6)
    for w in range(B):
        feats, rows, px = [], [], []
        for sem in torch.unique(labels[w]):
            sel = labels[w] == sem
            pts = x[w, sel]
            px.append(pts)
            lo, hi = pts.min(dim=0).values, pts.max(dim=0).values
            param_def[w, int(sem)] = torch.cat([(lo + hi) / 2.0, (hi - lo) / 2.0])
            f = per_point[w, sel]
            m = f.mean(dim=0)
            feats.append(m)
            rows.append(torch.cat([f, m.unsqueeze(0).expand(f.shape[0], -1)], dim=-1))
        k = len(feats)
        padded = torch.zeros(max_parts, C, dtype=per_point.dtype)
        padded = torch.cat([torch.stack(feats), padded[k:]], dim=0)
        mask[w, :k] = 1
        target_part_f.append(padded)
        re_in.append(torch.cat(rows, dim=0))
        part_x.append(px)
    return torch.stack(target_part_f), torch.stack(re_in), mask, part_x, param_def


def get_shape(A, param, default_param, weight):
    """dataset/dataset_utils.py:691-726 (no connectivity, no param_init)."""
    B, Pn, D = param.shape
    A = A.reshape(B * Pn, -1, D)
    p = weight * param.reshape(B * Pn, D, 1) + default_param.reshape(B * Pn, D, 1)
    return torch.bmm(A, p).reshape(B, Pn, -1, 3)


def get_symmetric(pc):
    return torch.cat([-pc[:, :, :1], pc[:, :, 1:2], pc[:, :, 2:3]], dim=2)


NN_TIE_STATS = {}          # filled by the index checks below; reset / read by the parity tests


def _nn_stat(name, over, exact, ratio):
    st = NN_TIE_STATS.setdefault(name, {"overridden": 0, "exact_ties": 0, "near_ties": 0, "max_over_bound": 0.0})
    st["overridden"] += int(over.sum())
    st["exact_ties"] += int((over & exact).sum())
    st["near_ties"] += int((over & ~exact).sum())
    if bool(over.any()):
        st["max_over_bound"] = max(st["max_over_bound"], float(ratio[over].max()))


def check_nn_choice(P_q, P_c, j_given, j_own, delta_q, delta_c, name):
    """NN indices chosen by another implementation from its own copy q of one point set (the HIP
    step's fp32 deformed shape), checked against the nearest neighbours here: for query i the
    given candidate j must satisfy |P_q[i] - P_c[j]| <= (d_i + dq_i + dc)(1 + 4u) + dq_i + dc,
    with d_i = |P_q[i] - P_c[own]|, dq_i = |q_i - P_q[i]| when the queries are the copied set,
    dc = max_k |q_k - P_c[k]| when the candidates are (the triangle inequality around the other
    implementation's own argmin, plus its fp32 distance rounding). P_q [B, n, 3], P_c [B, m, 3]
    float64; j_given / j_own [B, n] int; delta_q [B, n] or 0; delta_c [B] or 0."""
    bi = torch.arange(P_q.shape[0]).unsqueeze(1)
    e = (P_q - P_c[bi, j_given]).norm(dim=-1)
    d = (P_q - P_c[bi, j_own]).norm(dim=-1)
    dq = delta_q if torch.is_tensor(delta_q) else torch.zeros_like(d)
    dc = delta_c.unsqueeze(1) if torch.is_tensor(delta_c) else torch.zeros_like(d)
    # the copy's own deviation must be small next to the point sets' extent (the bound
    # grows with it, so it may not be what makes a wrong index acceptable)
    ext = torch.maximum(P_q.abs().amax(), P_c.abs().amax()) + 1e-30
    worst = float(torch.maximum(dq.max(), dc.max()) / ext) if dq.numel() else 0.0
    if worst > NN_DEV_TOL:
        raise AssertionError(f"NN tie check ({name}): the other implementation's copy deviates {worst:.3e} of the "
                             f"point sets' extent (> {NN_DEV_TOL:.0e}): its points are wrong, not its tie choice")
    bound = (d + dq + dc) * (1 + 4 * U32) + dq + dc
    over = j_given != j_own
    if bool((e > bound).any()):
        raise AssertionError(f"given NN index ({name}) is {float((e - bound).max()):.3e} farther than the "
                             "fp32 deviation bound around the nearest point: not a near-tie")
    _nn_stat(name, over, e == d, (e - d) / (bound - d + 1e-300))


class _OracleNN(torch.autograd.Function):
    """Chamfer primitive on the C oracle (values and idx bit-exact to the contract).

    q1 (optional): another copy of p1 (e.g. the HIP step's fp32 deformed shape) from which the
    NN indices of both directions are taken instead of p1's own. The distances are then those
    of p1 / p2 at these indices, each checked (check_nn_choice) to be the minimum up to the two
    copies' deviation, so a parity test compares gradients routed to the same points."""

    @staticmethod
    def forward(ctx, p1, p2, q1=None):
        a, b = p1.detach().float().numpy(), p2.detach().float().numpy()
        d1, d2, i1, i2 = nn_ref.nn_fwd(a, b)
        if q1 is not None:
            _, _, g1, g2 = nn_ref.nn_fwd(np.ascontiguousarray(q1.detach().float().numpy()), b)
            P1, P2 = p1.detach().double(), p2.detach().double()
            dev = (q1.detach().double() - P1).norm(dim=-1)                  # [B, n]
            t = lambda v: torch.from_numpy(np.asarray(v)).long()           # noqa: E731
            check_nn_choice(P1, P2, t(g1), t(i1), dev, 0, "p1 -> p2")
            check_nn_choice(P2, P1, t(g2), t(i2), 0, dev.amax(dim=1), "p2 -> p1")
            i1, i2 = g1, g2
            bi = torch.arange(P1.shape[0]).unsqueeze(1)
            d1 = ((p1.detach() - p2.detach()[bi, t(i1)]) ** 2).sum(-1).numpy()
            d2 = ((p2.detach() - p1.detach()[bi, t(i2)]) ** 2).sum(-1).numpy()
        ctx.save_for_backward(p1, p2)
        ctx.idx = (i1, i2)
        return torch.from_numpy(np.asarray(d1)).to(p1.dtype), torch.from_numpy(np.asarray(d2)).to(p1.dtype)

    @staticmethod
    def backward(ctx, g1, g2):
        p1, p2 = ctx.saved_tensors
        i1, i2 = ctx.idx
        r1, r2 = nn_ref.nn_bwd(p1.detach().float().numpy(), p2.detach().float().numpy(),
                               g1.float().numpy(), g2.float().numpy(), i1, i2)
        return torch.from_numpy(r1).to(p1.dtype), torch.from_numpy(r2).to(p2.dtype), None


def chamfer_costs(p1, p2, q1=None):
    """Shape_Measure ChamferLoss stand-in: squared NN distances (cost1 [B,n], cost2 [B,m]).
    q1: optional index source for p1 (see _OracleNN)."""
    return _OracleNN.apply(p1, p2, q1)


def chamfer_distance2(p1, p2, q1=None):
    c1, c2 = chamfer_costs(p1, p2, q1)
    return c1.mean(dim=1) + c2.mean(dim=1)


def compute_cm_loss(source_p, target_p, target_part, mask=None, np_per_part=1024, source_q=None):
    """source_q: optional NN index source for source_p (the same shape; see _OracleNN)."""
    if mask is None:
        return chamfer_distance2(source_p, target_p, source_q)
    n_valid = mask.sum(1) * np_per_part
    q = (lambda sl: None) if source_q is None else (lambda sl: source_q[sl])
    full, part = [], []
    for b in range(source_p.shape[0]):
        sl = (slice(b, b + 1), slice(0, int(n_valid[b].item())))
        full.append(chamfer_distance2(source_p[sl], target_p[b:b + 1], q(sl)))
        lp = []
        for i, tp in enumerate(target_part[b]):
            sl = (slice(b, b + 1), slice(i * np_per_part, (i + 1) * np_per_part))
            lp.append(chamfer_distance2(source_p[sl], tp.unsqueeze(0), q(sl)))
        part.append(torch.stack(lp).mean())
    return torch.stack(full).mean(), torch.stack(part).mean()


def residual_retrieval_loss(x, x_source, residuals, mask, np_per_part=1024, source_q=None):
    """source_q: optional NN index source for x_source (see _OracleNN)."""
    n_valid = mask.sum(1) * np_per_part
    nns = []
    for b in range(x.shape[0]):
        src = x_source[b, :int(n_valid[b].item())].detach()
        xs = x[b].detach().float().numpy()
        _, idx = nn_ref.nn_dir(xs, src.float().numpy())
        if source_q is not None:
            qb = source_q[b, :int(n_valid[b].item())].detach()
            own = idx
            _, idx = nn_ref.nn_dir(xs, np.ascontiguousarray(qb.float().numpy()))
            dc = (qb.double() - src.double()).norm(dim=-1).amax().reshape(1)
            check_nn_choice(x[b:b + 1].detach().double(), src.double().unsqueeze(0),
                            torch.from_numpy(idx).long().unsqueeze(0), torch.from_numpy(own).long().unsqueeze(0),
                            0, dc, "kNN x -> out")
        nns.append(src[torch.from_numpy(idx).long()])
    nn = torch.stack(nns)
    res = x + residuals - nn
    return res.abs().sum(-1).mean(), residuals.abs().sum(-1).mean()


def pc_consistency(a, b):
    d = a - b
    return (d * d).sum(-1).mean()


def pc_consistency_weighted(a, b, mask):
    d = a - b
    per = (d * d).sum(-1).mean(-1)           # [B, P]
    return (per * mask).sum() / mask.sum()


def regularization_param(params_full, mask_part):
    """loss/regularization_loss.py:49-53: boolean-indexed rows, then the mean L2 norm."""
    m = mask_part.reshape(-1).bool()
    return torch.norm(params_full.reshape(-1, 6)[m], p=2, dim=-1).mean()


def contrast_loss(tgt_part_f, src_f, src_labels, rank=0, gathered_src=None):
    B, Pn = src_f.shape[0], src_f.shape[1]
    t = F.normalize(tgt_part_f.reshape(B * Pn, -1), dim=-1, p=2)
    s = F.normalize(src_f.reshape(B * Pn, -1), dim=-1, p=2)
    labels = B * Pn * rank + torch.arange(B * Pn)
    labels[src_labels.reshape(-1) == -1] = -1
    s_all = s if gathered_src is None else gathered_src
    scale = torch.tensor(math.log(1 / 0.07)).exp()
    return F.cross_entropy(scale * t @ s_all.t(), labels, ignore_index=-1)


# ----------------------------------------------------------------------------
# the train step
# ----------------------------------------------------------------------------

LOSS_WEIGHTS_KEYS = ("use_chamfer_loss", "use_chamfer_part_loss", "use_contrast_loss",
                     "use_symmetry_loss", "use_residuals_reg", "use_recon")


def train_forward(params, batch, cfg, training=True, epoch=0):
    """engine/train.py:204-335 on a synthetic batch dict (numpy/torch CPU tensors).

    Returns (loss_all, terms dict). params: dict module -> state_dict (tensors may
    require grad). BN running stats inside params are updated in place (training).
    """
    P_max = cfg["MAX_NUM_PARTS"]
    emb = params["embedding_layer"]["weight"]
    src_idx = batch["src_index"]                          # [B,P] (already -1 -> last source)
    src_pts = batch["src_points"][src_idx]                # [B,P,1024,3]
    mats = batch["src_mats"][src_idx]                     # [B,P,3072,6]
    src_sem_f = emb[batch["src_sem"][src_idx]]
    tgt_sem_f = emb[batch["tgt_sem"]]
    x = batch["x"]
    if cfg.get("complementme", False):
        x = x.clone()
        x[:, :, 2] = -x[:, :, 2]
    B = x.shape[0]

    pool = batch.get("_pool_idx", {})      # optional max-pool winners to follow (see max_pool)
    pvals = batch.get("_pool_gpu", {})     # ... and the values they were chosen from
    prec = {"src_encoder_all": {}, "target_encoder_full": {}}
    codes, src_pp = target_encoder(params["src_encoder_all"], src_pts, src_sem_f, True, training,
                                   pool.get("src_encoder_all"), prec["src_encoder_all"], pvals.get("src_encoder_all"))
    rin = torch.cat([codes.unsqueeze(2).expand(-1, -1, src_pp.shape[-1]), src_pp], dim=1)
    recon_src = residual_net(params["recon_decoder_src"], rin.permute(0, 2, 1), training)
    recon_src = recon_src.reshape(B, P_max, -1, 3)

    tcode, pp = target_encoder(params["target_encoder_full"], x, tgt_sem_f, False, training,
                               pool.get("target_encoder_full"), prec["target_encoder_full"],
                               pvals.get("target_encoder_full"))
    pp = pp.permute(0, 2, 1)
    part_f, re_in, mask, part_x, param_def = get_part(pp, batch["labels"], x, P_max)
    N = pp.shape[1]
    recon_full = residual_net(params["recon_decoder_full"],
                              torch.cat([pp, tcode.unsqueeze(1).expand(-1, N, -1)], dim=-1), training)
    re_res = residual_net(params["re_residual_net_full"], re_in, training)
    codes = codes.reshape(B, P_max, -1)
    prm = deform_net(params["param_decoder_full"], tcode, codes, training=training)
    out = get_shape(mats, prm, param_def, cfg["alpha"]).reshape(B, -1, 3)

    T = OrderedDict()
    # optional NN index source: the HIP step's fp32 deformed shape (see _OracleNN)
    oq = batch.get("_nn_out")
    use_param = cfg.get("use_param_loss", 0.0) > 0.0
    if use_param:
        T["param_loss"] = regularization_param(prm, mask)
    T["cd_loss_full"], T["cd_loss_part"] = compute_cm_loss(out, x, part_x, mask, source_q=oq)
    T["contrast_loss"] = contrast_loss(part_f, codes, batch["src_labels"])
    T["ref_cd_loss_full"], T["ref_cd_loss_part"] = compute_cm_loss(
        get_symmetric(out), x, part_x, mask, source_q=None if oq is None else get_symmetric(oq))
    if epoch > cfg["init_p_m_loss"]:
        T["re_reg_loss_full"], T["reg_loss_full"] = residual_retrieval_loss(x, out.detach(), re_res, mask,
                                                                            source_q=oq)
    T["recon_loss_full"] = pc_consistency(recon_full, x)
    T["recon_loss_src"] = pc_consistency_weighted(recon_src, src_pts, mask)
    loss = T["param_loss"] * cfg["use_param_loss"] if use_param else 0.0
    loss = (loss + T["cd_loss_full"] * cfg["use_chamfer_loss"] + T["cd_loss_part"] * cfg["use_chamfer_part_loss"]
            + T["contrast_loss"] * cfg["use_contrast_loss"] + T["ref_cd_loss_full"] * cfg["use_symmetry_loss"])
    if "re_reg_loss_full" in T:
        loss = loss + T["re_reg_loss_full"] * cfg["use_residuals_reg"] + T["reg_loss_full"] * cfg["use_residuals_reg"] * 0.01
    loss = loss + T["recon_loss_full"] * cfg["use_recon"] + T["recon_loss_src"] * cfg["use_recon"]
    T["all_loss"] = loss
    T["_out"] = out
    T["_params"] = prm
    T["_pool"] = prec
    return loss, T


TRAINED_MODULES = ("target_encoder_full", "param_decoder_full", "re_residual_net_full",
                   "recon_decoder_full", "src_encoder_all", "recon_decoder_src")


def trainable(params):
    """The tensors that the reference hands to Adam (embedding excluded) in its order."""
    out = []
    for mod in TRAINED_MODULES:
        for k, v in params[mod].items():
            if v.dtype.is_floating_point and not (k.endswith("running_mean") or k.endswith("running_var")):
                out.append((mod, k, v))
    return out


# ----------------------------------------------------------------------------
# inference (engine/vis.py:118-256, batched)
# ----------------------------------------------------------------------------

def infer(params, batch, cfg, chunk=512, retrieved=None):
    """Retrieval + deformation in eval mode. batch holds src_points/src_mats/src_sem (the whole DB),
    x, labels, tgt_sem. Returns retrieved [B,P] (-1 for empty slots), top-2 gap, the similarity
    matrix [B,P,S], params, out, cd [B]. retrieved (optional, [B,P]): deform these sources instead
    of the argmax (the test deforms the GPU's picks where a near-tie flipped one)."""
    with torch.no_grad():
        emb = params["embedding_layer"]["weight"]
        pts, sem = batch["src_points"], batch["src_sem"]
        codes = []
        for s in range(0, pts.shape[0], chunk):
            c, _ = target_encoder(params["src_encoder_all"], pts[s:s + chunk].unsqueeze(1),
                                  emb[sem[s:s + chunk]].unsqueeze(1), True, training=False)
            codes.append(c)
        codes = F.normalize(torch.cat(codes), dim=-1, p=2)
        x = batch["x"]
        B = x.shape[0]
        P = cfg["MAX_NUM_PARTS"]
        tcode, pp = target_encoder(params["target_encoder_full"], x, emb[batch["tgt_sem"]], False, training=False)
        part_f, _, mask, _, _ = get_part(pp.permute(0, 2, 1), batch["labels"], x, P)
        sim = F.normalize(part_f, dim=-1, p=2) @ codes.t()
        top2 = sim.topk(2, dim=-1).values
        if retrieved is None:
            retrieved = torch.where(mask > 0, sim.argmax(-1), torch.full((B, P), -1, dtype=torch.long))
        else:
            retrieved = torch.where(mask > 0, retrieved.long(), torch.full((B, P), -1, dtype=torch.long))
        idx = torch.where(retrieved < 0, retrieved + pts.shape[0], retrieved)
        prm = deform_net(params["param_decoder_full"], tcode, codes[idx], training=False)
        out = get_shape(batch["src_mats"][idx], prm, torch.zeros_like(prm), cfg["alpha"]).reshape(B, -1, 3)
        cd = chamfer_distance2(out, x)
        return {"retrieved": retrieved, "sim_top2_gap": top2[..., 0] - top2[..., 1], "sim": sim, "params": prm,
                "out": out, "cd": cd}
