"""The reference entry point as a multi-rank job: engine/train.py main() under
torch.distributed.run, world 2, gloo (cfg["dist_backend"]; both ranks on the one GPU of the
test box — RCCL needs one GPU per rank), through tests/dist_main_worker.py.

Per mode (eager DataParallelStep; HIP-graph replay with the collectives between the captured
segments; graph replay + SyncBN): 2 epochs x 2 iterations from the pseudo-label loader, each
rank on its own shard. Checked: exit status 0; the trained parameters are finite and bitwise
identical on both ranks (the gradient all-reduce); the BN running statistics are identical
across the ranks with SyncBN and differ without it (each rank normalises with its own shard's
statistics); rank 0 wrote one checkpoint per epoch, loadable with weights_only=True; the
StepLR schedule stepped once per epoch; the scalar log holds finite losses."""
import json
import math
import os
import socket
import subprocess
import sys

import pytest
import torch

from conftest import PKG_DIR, ROOT

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(400)
@pytest.mark.parametrize("mode", ["eager", "graph", "graph_sync_bn"])
def test_train_main_two_ranks(dev, tmp_path, mode):
    with open(os.path.join(PKG_DIR, "config", "config_train_test.json")) as f:
        cfg = json.load(f)
    log = tmp_path / "log"
    cfg.update(device="cuda", dist_backend="gloo", epochs=2, save_epoch=1, batch_size=2, num_points=1024,
               num_targets=4, log_every=1, log_path=str(log), cuda_graph=mode != "eager",
               sync_bn=mode == "graph_sync_bn")
    os.makedirs(log)
    cpath = tmp_path / "cfg.json"
    cpath.write_text(json.dumps(cfg))
    out = tmp_path / "out"
    os.makedirs(out)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "dist_main_worker.py"), str(cpath), str(out)]
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=360)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-6000:])
    r = [json.loads((out / f"rank{i}.json").read_text()) for i in range(2)]
    assert r[0]["finite"] and r[1]["finite"]
    assert r[0]["params"] == r[1]["params"], "the ranks' parameters diverged"
    if mode == "graph_sync_bn":
        assert r[0]["buffers"] == r[1]["buffers"], "SyncBN: the ranks' BN statistics differ"
    else:
        assert r[0]["buffers"] != r[1]["buffers"], "without SyncBN each rank keeps its own shard's statistics"
    if mode != "eager":
        assert r[0]["graphs"] >= 1
    assert r[0]["lr"] == cfg["learning_rate"] * cfg["lr_decay"] ** (2 // cfg["lr_stepsize"])
    for e in range(2):
        sd = torch.load(log / f"checkpoint_{e:04d}.pth", map_location="cpu", weights_only=True)
        assert set(sd) >= {"target_encoder_full", "param_decoder_full", "src_encoder_all"}
    vals = []
    if (log / "scalars.jsonl").exists():
        vals = [json.loads(line)["value"] for line in (log / "scalars.jsonl").read_text().splitlines()]
        assert vals and all(math.isfinite(v) for v in vals)
    print(f"{mode}: ranks agree ({r[0]['params'][:12]}), {len(vals)} logged scalars")
