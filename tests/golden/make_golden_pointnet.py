"""Golden vectors for PointNetEncoder FROM THE REFERENCE ITSELF (run here,
where /root/reference exists; never on the GPU box).

  python tests/golden/make_golden_pointnet.py

Imports network/pointnet/pointnet_utils.py of the reference (torch + numpy only), loads the
deterministic parameters of oracle.pointnet_ref.make_params with strict=True (which also pins
the state_dict key list), runs forward in training mode and backward of a seeded scalar loss
for each case of oracle.pointnet_ref.CASES, and writes inputs + outputs + gradients (full for
small tensors; norm + 256 seeded samples for large ones) to tests/golden/pointnet.npz.
"""
import os
import sys

import numpy as np
import torch

os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(1, os.path.join(REF, "network", "pointnet"))

import pointnet_utils as ref  # noqa: E402  (reference)
from oracle import pointnet_ref  # noqa: E402

SAMPLE = 256


def main():
    out = {}
    for ci, (name, B, D, N, gf, ft) in enumerate(pointnet_ref.CASES):
        torch.manual_seed(0)
        m = ref.PointNetEncoder(global_feat=gf, feature_transform=ft, channel=D)
        m.load_state_dict(pointnet_ref.make_params(D, ft, seed=10 + ci), strict=True)
        m.train()
        x, _ = pointnet_ref.case_inputs(B, D, N, seed=100 + ci)
        xt = torch.from_numpy(x).requires_grad_(True)
        o, trans, trans_feat = m(xt)
        loss = pointnet_ref.case_loss(o, trans, trans_feat, rng_seed=1000 + ci)
        loss.backward()
        out[f"{name}/x"] = x
        out[f"{name}/out"] = o.detach().numpy()
        out[f"{name}/trans"] = trans.detach().numpy()
        if trans_feat is not None:
            out[f"{name}/trans_feat"] = trans_feat.detach().numpy()
        out[f"{name}/loss"] = np.float64(loss.item())
        out[f"{name}/dx"] = xt.grad.numpy()
        rng = np.random.Generator(np.random.PCG64(7))
        for k, p in m.named_parameters():
            g = p.grad.detach().numpy().reshape(-1)
            if g.size <= 20000:
                out[f"{name}/grad/{k}"] = g
            else:
                idx = rng.choice(g.size, SAMPLE, replace=False).astype(np.int64)
                out[f"{name}/gnorm/{k}"] = np.float64(np.linalg.norm(g.astype(np.float64)))
                out[f"{name}/gidx/{k}"] = idx
                out[f"{name}/gval/{k}"] = g[idx]
        # running statistics after the step (BN momentum update)
        for k, v in m.state_dict().items():
            if k.endswith("running_mean") or k.endswith("running_var"):
                out[f"{name}/state/{k}"] = v.numpy()
    np.savez_compressed(os.path.join(HERE, "pointnet.npz"), **out)
    print("wrote", len(out), "arrays")


if __name__ == "__main__":
    main()
