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
    lines = [x for x in r.stdout.splitlines() if x.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout  # gloo's rendezvous chatter goes to stderr
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


_STEADY_WORKER = r"""
import os, sys, time
import torch
import torch.distributed as dist
sys.path.insert(0, os.environ["ROOT"])
torch.cuda.synchronize = lambda *a, **k: None  # CPU rehearsal: nothing to wait for
import bench
dist.init_process_group("gloo")
rank = dist.get_rank()
calls = [0]
def step():  # a step holding a collective (as the encoder leg's symbol-stream gather does)
    calls[0] += 1
    if rank == 1:
        time.sleep(0.004)  # rank 1's steps are slower: a time-bounded pre-warm would call fewer of them
    t = torch.ones(1)
    dist.all_reduce(t)
    assert int(t.item()) == dist.get_world_size()
el = bench.timed_steady(step, 3, "cpu", prewarm_ms=40.0)
c = torch.tensor([calls[0]])
dist.all_reduce(c, op=dist.ReduceOp.MAX)
assert int(c.item()) == calls[0], (rank, calls[0], int(c.item()))
print("OK", rank, calls[0], el)
dist.destroy_process_group()
"""


def test_timed_steady_prewarm_agrees_across_ranks():
    """bench.timed_steady pre-warms a secondary leg's step a number of times every rank agrees on:
    the encoder leg's step holds collectives, so ranks whose steps run at different speeds must still
    call it equally often (gloo, world 2, rank 1 deliberately slower)."""
    import socket
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    procs = [subprocess.Popen([sys.executable, "-c", _STEADY_WORKER], cwd=ROOT, stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True,
                              env=_env(ROOT=ROOT, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                                       MASTER_PORT=str(port)))
             for r in range(2)]
    outs = [p.communicate(timeout=240) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
        assert any(x.startswith("OK") for x in o.splitlines()), o
