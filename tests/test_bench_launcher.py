"""bench.py's own multi-GPU launch (`--gpus N` without a launcher environment), on
the CPU: the script starts N fresh rank processes with RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_* set, they rendezvous (gloo here), and a rank that dies ends
the whole run with its status instead of leaving the others blocked."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n, extra_env=None, timeout=180):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n),
                           "--rank-check"], env=env, cwd="/tmp", capture_output=True, text=True,
                          timeout=timeout)


@pytest.mark.parametrize("n", [2, 4])
def test_gpus_n_launches_n_ranks(n):
    r = _run(n)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 alone prints
    out = json.loads(lines[0])
    assert out["world"] == n
    assert out["ranks"] == [[i, i, n] for i in range(n)]


def test_failed_rank_ends_the_run():
    r = _run(2, {"VAESNE_RANK_CHECK_FAIL": "1"}, timeout=120)
    assert r.returncode != 0
    assert not any(ln.startswith("{") for ln in r.stdout.splitlines())


def test_single_gpu_does_not_spawn():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1",
                        "--rank-check"], cwd="/tmp", capture_output=True, text=True, timeout=120,
                       env={k: v for k, v in os.environ.items() if k != "WORLD_SIZE"})
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1]) == {"world": 1, "ranks": [[0, 0, 1]]}
