"""bench.py's N > 1 path end to end on the one GPU of a test box: `--gpus 2 --dist-backend gloo`
launches two ranks through torch.distributed.run (both on GPU 0), replays the data-parallel step
as segmented HIP graphs (the contrastive all_gather between the segments, the gradient
all-reduce after them) and prints ONE JSON line with the whole-job rate. The driver's scaling
run is the same code with RCCL and one GPU per rank; the rate here means nothing."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(400)
def test_bench_two_ranks_gloo(dev):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo", "--steps", "3",
           "--warmup", "1", "--batch", "4", "--no-extras", "--no-cpu-baseline", "--no-breakdown",
           "--no-all-slots-rate", "--no-k16-rate", "--no-loader-rate"]
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=360)
    assert p.returncode == 0, p.stderr[-5000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-3000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2" and d["scaling"] == "weak"
    assert d["step_mode"] == "hip_graph"
    assert d["value"] > 0 and d["config"]["global_batch"] == 8
    print(lines[0][:300])
