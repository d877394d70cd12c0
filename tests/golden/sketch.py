"""How the golden train-step files store a gradient tensor (shared by make_golden.py, which
writes them, and tests/test_oracle_golden.py, which applies the same reduction to the oracle's
gradients). Data layout only — no reference code."""
import numpy as np


def grad_sketch(name, g, full_max=16384, nsample=2048, nproj=16):
    """Whole when the tensor has <= full_max elements; otherwise its row sums (over every dim but
    the first), column sums (over the first dim), nsample elements at PCG64(name)-drawn flat
    indices and nproj Gaussian projections (each a dot product with the whole tensor, so a
    deviation anywhere moves them). g: torch tensor; returns float64 numpy arrays."""
    g = g.detach().double()
    g = g.reshape(g.shape[0], -1) if g.dim() > 1 else g.reshape(-1, 1)
    if g.numel() <= full_max:
        return {"full": g.numpy()}
    h = int.from_bytes(name.encode(), "little") % (2 ** 63)
    rng = np.random.Generator(np.random.PCG64([h % (2 ** 32), h >> 32]))
    flat = g.reshape(-1).numpy()
    idx = rng.integers(0, flat.size, size=nsample).astype(np.int32)
    proj = rng.standard_normal(size=(nproj, flat.size))
    return {"rows": g.sum(1).numpy(), "cols": g.sum(0).numpy(), "idx": idx, "sample": flat[idx],
            "proj": proj @ flat}


STEP_CASES = {
    # file: (cfg overrides, parts per target of the 2-sample batch)
    "train_step.npz": ({}, [3, 2]),
    # the two reference keys that are off in the shipped config: the parameter regulariser
    # (engine/train.py:281-283) and the ComplementMe z-flip of the targets (:192-194)
    "train_step_param.npz": ({"use_param_loss": 1.0, "complementme": True}, [4, 2]),
}
