"""Whole-step parity checks shared by the train-step GPU tests (tests/test_train_step_gpu.py,
tests/test_fullsize_gpu.py): the HIP step's loss terms and EVERY parameter gradient tensor
against the float64 oracle (oracle/ured_ref.py, itself pinned elementwise to the reference's
composed step by tests/test_oracle_golden.py).

Tolerances (SURVEY §8(d) for the loss):
  * every loss term within LOSS_RTOL = 1e-5 relative;
  * every gradient tensor: ||g - g_ref|| / ||g_ref|| <= max(GRAD_REL = 1e-3, 3 x the same oracle's
    own fp32 deviation) and max |g - g_ref| <= max(GRAD_ELEM = 1e-2, 3 x the fp32 oracle's) x
    max |g_ref| (elementwise, so a permuted or misrouted row — which keeps the norm — fails).
    The fp32 floor: the oracle re-run in fp32 (the reference's own arithmetic width) shows how
    far fp32 accumulation alone moves each gradient from float64; a few tensors sit above 1e-3
    there (BatchNorm-backward cancellations in long column sums; max-pool / NN near-ties that
    fp32 rounding resolves the other way), and the HIP step is held to 3x that, not to a
    tolerance tuned to the HIP result;
  * exactly-zero true gradients (a conv bias feeding a training-mode BatchNorm; the attention
    key bias, which softmax cancels) are rounding noise on both sides: bounded against the
    matching weight gradient instead.
"""
import torch

LOSS_RTOL = 1e-5
GRAD_REL = 1e-3
GRAD_ELEM = 1e-2

TRAINED = ("target_encoder_full", "param_decoder_full", "re_residual_net_full", "recon_decoder_full",
           "src_encoder_all", "recon_decoder_src")
ENC_BN_FED = ("mlp1.0.bias", "mlp1.3.bias", "mlp2.0.bias", "mlp2.3.bias", "mlp2.6.bias", "fuse_sem.0.bias",
              "per_point_out.0.bias")


ENCODERS = ("src_encoder_all", "target_encoder_full")


class ParityReport(UserWarning):
    """Carries the parity tests' measured numbers (tie gaps, loss-term deviations, worst gradient
    tensors) into pytest's warnings summary, so a quiet (-q) run still shows them."""


def report(line):
    import warnings
    print(line)
    warnings.warn(line.strip(), ParityReport, stacklevel=2)


def record_pools(models, on=True):
    for name in ENCODERS:
        models[name].record_pool = on


def gpu_pool_choices(models, batch, unique):
    """The HIP step's max-pool winners ({encoder: [groups, 1024] point index within the group}),
    in the oracle's grouping: every source slot of the batch (unique-source encoding runs one
    group per distinct part; slot s took the winners of part inverse[s])."""
    out = {}
    for name in ENCODERS:
        idx = models[name].last_pool_idx
        assert idx is not None, f"{name}: forward ran without record_pool"
        if name == "src_encoder_all" and unique:
            idx = idx[batch["src_unique"].inverse]
        out[name] = idx.cpu()
    return out


def gpu_pool_values(models, batch, unique):
    """{encoder: gpu_h} for ured_ref.max_pool: gpu_h(pidx [groups, 1024]) -> the HIP step's pooled
    activation relu(y * scale + shift) (fp32, as its kernels compute it) at point pidx[g, c] of
    group g, channel c, in the oracle's grouping (unique-source encoding: slot s reads the
    distinct part inverse[s])."""
    out = {}
    for name in ENCODERS:
        y, sc, sh, n = models[name].last_pool_vals
        y, sc, sh = y.detach().cpu(), sc.detach().cpu(), sh.detach().cpu()
        grp = None
        if name == "src_encoder_all" and unique:
            grp = batch["src_unique"].inverse.cpu()

        def gpu_h(pidx, y=y, sc=sc, sh=sh, n=n, grp=grp):
            G, C = pidx.shape
            g = torch.arange(G).unsqueeze(1) if grp is None else grp.unsqueeze(1)
            rows = g * n + pidx.long()
            v = y[rows, torch.arange(C).unsqueeze(0)]
            return torch.relu(torch.addcmul(sh.unsqueeze(0), v, sc.unsqueeze(0))).double()
        out[name] = gpu_h
    return out


def tie_report(pool_rec, label=""):
    """Prints the max-pool and NN tie statistics of one oracle run (ured_ref.max_pool records,
    ured_ref.NN_TIE_STATS): winners taken from the HIP step, exact ties (equal values) vs near-ties,
    and the largest gap, absolute / relative to the channel / relative to its fp32 bound."""
    from oracle import ured_ref
    parts = []
    for n in ENCODERS:
        r = pool_rec[n]
        if "overridden" in r:
            parts.append(f"{n}: {r['overridden']} overridden ({r['exact_ties']} exact ties, {r['near_ties']} near-ties), "
                         f"max gap {r['max_gap']:.2e} ({r['max_gap_rel']:.2e} of the channel max, "
                         f"{r['max_gap_over_bound']:.2f} of the fp32 bound; HIP activation deviation "
                         f"{r['max_dev_rel']:.1e} of the layer scale)")
    for k, st in sorted(ured_ref.NN_TIE_STATS.items()):
        parts.append(f"NN {k}: {st['overridden']} overridden ({st['exact_ties']} exact, {st['near_ties']} near), "
                     f"max {st['max_over_bound']:.2f} of the bound")
    report(f"\n{label} ties: " + "; ".join(parts))


def same_pools(choices, oracle_pool):
    """True when the GPU's winners are the oracle's own argmax everywhere."""
    return all(torch.equal(choices[n].long(), oracle_pool[n]["argmax"].long().cpu()) for n in ENCODERS)


def zero_true_grad(mod, k):
    if mod in ("target_encoder_full", "src_encoder_all") and k in ENC_BN_FED:
        return True
    return k.endswith("in_proj_k.bias")


def check_loss_terms(got, ref, label=""):
    """got/ref: {term: float}. Prints every term's relative deviation; asserts LOSS_RTOL."""
    assert set(got) == set(ref), (sorted(got), sorted(ref))
    dev = {k: abs(got[k] - ref[k]) / max(abs(ref[k]), 1e-30) for k in ref}
    report(f"\n{label} loss-term rel dev: " + ", ".join(f"{k} {v:.1e}" for k, v in sorted(dev.items())))
    for k, v in dev.items():
        assert v <= LOSS_RTOL, f"{label} {k}: {got[k]!r} vs {ref[k]!r} (rel {v:.2e} > {LOSS_RTOL})"
    return dev


def _devs(g, r):
    return ((g - r).norm().item() / max(r.norm().item(), 1e-30),
            (g - r).abs().max().item() / max(r.abs().max().item(), 1e-30))


def check_grads(models, ref_grads, label="", ref32=None, grad_rel=GRAD_REL, grad_elem=GRAD_ELEM, floor_mult=3.0):
    """models: the HIP step's modules (after backward); ref_grads: {(module, name): float64 CPU
    tensor or None}; ref32: the same oracle's gradients from an fp32 run (the per-tensor noise
    floor) or None. Every trained parameter is compared as a whole tensor."""
    rows, n, floored, nbig = [], 0, 0, 0
    for mod in TRAINED:
        params = dict(models[mod].named_parameters())
        for k, p in params.items():
            r = ref_grads[(mod, k)]
            if r is None:
                assert p.grad is None, f"{label} {mod}.{k} should get no gradient"
                continue
            assert p.grad is not None, f"{label} {mod}.{k} has no gradient"
            g = p.grad.detach().double().cpu()
            assert g.shape == r.shape, (mod, k, g.shape, r.shape)
            if zero_true_grad(mod, k):
                wr = ref_grads[(mod, k[:-5] + ".weight")].norm().item()
                assert g.norm().item() <= 1e-2 * wr + 1e-4 and r.norm().item() <= 1e-2 * wr + 1e-4, \
                    f"{label} {mod}.{k}: |g| {g.norm().item():.3e} |g_ref| {r.norm().item():.3e} vs |dW| {wr:.3e}"
                continue
            rel, elem = _devs(g, r)
            lim_rel, lim_elem, f32 = grad_rel, grad_elem, (0.0, 0.0)
            if ref32 is not None:
                f32 = _devs(ref32[(mod, k)].double(), r)
                lim_rel, lim_elem = max(lim_rel, floor_mult * f32[0]), max(lim_elem, floor_mult * f32[1])
                floored += int(lim_rel > grad_rel or lim_elem > grad_elem)
            rows.append((rel, elem, f"{mod}.{k}", f32, lim_rel, lim_elem))
            nbig += int(((g - r).abs() > 2e-3 * r.abs().max()).sum())
            n += 1
    rows.sort(key=lambda t: -t[0])
    report(f"{label} {n} gradient tensors ({floored} with an fp32 floor above {grad_rel:g}/{grad_elem:g}; "
          f"{nbig} elements off by > 2e-3 of their tensor's max); "
          f"worst rel-norm / elementwise dev [fp32 oracle's]: " +
          "; ".join(f"{name} {rel:.1e}/{elem:.1e} [{f[0]:.1e}/{f[1]:.1e}]" for rel, elem, name, f, _, _ in rows[:6]))
    bad = [(name, f"{rel:.2e}>{lr:.2e}" if rel > lr else "", f"{elem:.2e}>{le:.2e}" if elem > le else "")
           for rel, elem, name, _, lr, le in rows if rel > lr or elem > le]
    assert not bad, f"{label} gradient tensors off the oracle: {bad[:8]}"
    return n, rows
