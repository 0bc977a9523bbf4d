"""CPU: bench.py is the authority on the world size.

`python bench.py --gpus N` with no launcher around it starts N rank processes
itself (subprocesses with the torch.distributed.run environment, before any GPU
call) and its output is rank 0's one JSON line; under a launcher, --gpus must
equal WORLD_SIZE.  --launch-check exercises exactly that plumbing with a gloo
rendezvous and no GPU (the -m gpu test test_bench_gpus2_gloo runs the full
bench at --gpus 2)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env.update(kw)
    return env


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_flag_spawns_the_ranks(n):
    r = subprocess.run([sys.executable, "bench.py", "--gpus", str(n), "--launch-check"], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d == {"n_gpus": n, "world_size": n, "rank_sum": n * (n - 1) // 2, "backend": "gloo"}, d


def test_gpus_must_match_launcher_world():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--launch-check"], cwd=ROOT,
                       env=_env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=3" in r.stderr, (r.returncode, r.stderr[-2000:])
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "0", "--launch-check"], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
