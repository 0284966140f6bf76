"""bench.py --gpus N must start N ranks itself when no torch.distributed launcher wraps it
(the driver's multi-GPU run may call it either way). Rehearsed on CPU with gloo and no GPU
work: one JSON line from rank 0 carrying n_gpus == N."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(*args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + list(args), env=env, cwd=ROOT,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=240)
    return p


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_launches_n_ranks(n):
    p = run_bench("--gpus", str(n), "--steps", "3", "--warmup", "0", "--launcher-check")
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    lines = [ln for ln in p.stdout.decode().splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout.decode()
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["steps"] == 3 and d["launcher_check"]
    assert d["world_size_seen"] == n
    # N > 1 measures the target config by default: C5 (1B records) strong scaling
    assert d["workload"] == "c5"


def test_gpus_1_runs_in_process():
    p = run_bench("--gpus", "1", "--steps", "2", "--warmup", "0", "--launcher-check")
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    d = json.loads([ln for ln in p.stdout.decode().splitlines() if ln.startswith("{")][0])
    assert d["n_gpus"] == 1
    assert d["workload"] == "c2"  # the headline at N = 1 is BASELINE configs[1]


def test_world_size_mismatch_is_refused():
    p = run_bench("--gpus", "4", "--launcher-check", env_extra={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0
    assert b"WORLD_SIZE=2" in p.stderr
