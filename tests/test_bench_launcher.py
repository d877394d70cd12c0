"""bench.py's multi-rank launcher on CPU: `python bench.py --gpus 2` without torch.distributed.run
starts the two ranks itself, and the JSON line reports the world size the ranks actually formed
(--cpu-dry-run replaces the GPU step by a gloo all_reduce; the launch path is the real one)."""
import json
import os
import subprocess
import sys

from conftest import ROOT


def test_bench_gpus2_spawns_two_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3",
                        "--warmup", "1", "--cpu-dry-run"], capture_output=True, text=True, timeout=240, env=env,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 3 and out["dry_run"]
