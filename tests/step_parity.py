"""Whole-step parity checks shared by the train-step GPU tests (tests/test_train_step_gpu.py,
tests/test_fullsize_gpu.py): the HIP step's loss terms and EVERY parameter gradient tensor
against the float64 oracle (oracle/ured_ref.py, itself pinned elementwise to the reference's
composed step by tests/test_oracle_golden.py).

Tolerances (SURVEY §8(d) for the loss; the gradient bounds are set from measured fp32-vs-float64
deviations with margin, see DESIGN.md "Parity"):
  * every loss term within LOSS_RTOL = 1e-5 relative;
  * every gradient tensor: ||g - g_ref|| / ||g_ref|| <= GRAD_REL (1e-3) and
    max |g - g_ref| <= GRAD_ELEM * max |g_ref| (elementwise, so a permuted or misrouted row —
    which keeps the norm — fails);
  * exactly-zero true gradients (a conv bias feeding a training-mode BatchNorm; the attention
    key bias, which softmax cancels) are rounding noise on both sides: bounded against the
    matching weight gradient instead.
"""
import torch

LOSS_RTOL = 1e-5
GRAD_REL = 1e-3
GRAD_ELEM = 2e-3

TRAINED = ("target_encoder_full", "param_decoder_full", "re_residual_net_full", "recon_decoder_full",
           "src_encoder_all", "recon_decoder_src")
ENC_BN_FED = ("mlp1.0.bias", "mlp1.3.bias", "mlp2.0.bias", "mlp2.3.bias", "mlp2.6.bias", "fuse_sem.0.bias",
              "per_point_out.0.bias")


def zero_true_grad(mod, k):
    if mod in ("target_encoder_full", "src_encoder_all") and k in ENC_BN_FED:
        return True
    return k.endswith("in_proj_k.bias")


def check_loss_terms(got, ref, label=""):
    """got/ref: {term: float}. Prints every term's relative deviation; asserts LOSS_RTOL."""
    assert set(got) == set(ref), (sorted(got), sorted(ref))
    dev = {k: abs(got[k] - ref[k]) / max(abs(ref[k]), 1e-30) for k in ref}
    print(f"\n{label} loss-term rel dev: " + ", ".join(f"{k} {v:.1e}" for k, v in sorted(dev.items())))
    for k, v in dev.items():
        assert v <= LOSS_RTOL, f"{label} {k}: {got[k]!r} vs {ref[k]!r} (rel {v:.2e} > {LOSS_RTOL})"
    return dev


def check_grads(models, ref_grads, label="", grad_rel=GRAD_REL, grad_elem=GRAD_ELEM):
    """models: the HIP step's modules (after backward); ref_grads: {(module, name): float64 CPU
    tensor or None}. Every trained parameter is compared as a whole tensor."""
    rows, n = [], 0
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
            rn = r.norm().item()
            rel = (g - r).norm().item() / max(rn, 1e-30)
            elem = (g - r).abs().max().item() / max(r.abs().max().item(), 1e-30)
            rows.append((rel, elem, f"{mod}.{k}"))
            n += 1
    rows.sort(reverse=True)
    print(f"{label} {n} gradient tensors; worst rel-norm / elementwise dev: " +
          "; ".join(f"{name} {rel:.1e}/{elem:.1e}" for rel, elem, name in rows[:6]))
    bad = [(name, rel, elem) for rel, elem, name in rows if rel > grad_rel or elem > grad_elem]
    assert not bad, f"{label} gradient tensors off the oracle: {bad[:8]}"
    return n, rows
