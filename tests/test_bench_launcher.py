"""``bench.py --gpus N`` launches N ranks (CPU self-test, no GPU).

The driver runs ``python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N``; a
bare ``python bench.py --gpus N`` must do the same itself (spawning ``torch.distributed.run``
before any GPU call), and a launcher/``--gpus`` mismatch must fail instead of printing an N-GPU
line measured on fewer ranks.  ``--launch-check`` makes each rank rendezvous over gloo on
127.0.0.1, all-reduce its rank and exit, so the launcher path is exercised here without a GPU.
"""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env.update(kw)
    return env


@pytest.mark.timeout(240)
@pytest.mark.parametrize("n", [2, 3])
def test_bench_spawns_n_ranks(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--launch-check"], capture_output=True, text=True,
                       env=_env(), timeout=200)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == n
    assert out["rank_sum"] == out["expected"] == float(sum(range(n)))


@pytest.mark.timeout(120)
def test_bench_rejects_world_mismatch():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--launch-check"], capture_output=True, text=True,
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), timeout=100)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr
