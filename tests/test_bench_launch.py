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


_LEGS_WORKER = r"""
import datetime, json, os, sys, time
import torch
import torch.distributed as dist
sys.path.insert(0, os.environ["ROOT"])
import bench
mode = os.environ["MODE"]
dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=5))
rank, world = dist.get_rank(), dist.get_world_size()
rep = bench.Report(rank)
rep.out = {"value": 123.0}
legs = bench.Legs(rep, True, deadline_s=60.0)
rep.out["legs"] = legs.status

def all_gather():
    parts = [torch.empty(4) for _ in range(world)]
    dist.all_gather(parts, torch.full((4,), float(rank)))
    return [float(p[0]) for p in parts]

def p2p():  # the last rank fails before posting its push, as bench.py --gather-fault p2p-raise/-stall does
    if rank == world - 1:
        if mode == "stall":
            time.sleep(8.0)
        raise RuntimeError("injected")
    buf = torch.empty(4)
    for w in dist.batch_isend_irecv([dist.P2POp(dist.irecv, buf, group_peer=world - 1)]):
        w.wait()
    return "received"

t0 = time.time()
rep.out["ag"] = legs.run("ag", all_gather)
rep.out["p2p"] = legs.run("p2p", p2p)
rep.out["after"] = legs.run("after", all_gather)
rep.out["local"] = legs.run("local", lambda: 7, collective=False)
rep.out["elapsed"] = time.time() - t0
print("STATUS", rank, json.dumps(legs.status), flush=True)
rep.emit()
sys.stdout.flush()
os._exit(0)
"""


@pytest.mark.parametrize("mode", ["raise", "stall"])
def test_legs_fail_soft_p2p_peer(mode):
    """bench.Legs: at world 2 over gloo, the last rank fails its
    direct-push leg before posting (raising at once, or after stalling past the
    process group's 5 s timeout).  Rank 0's grouped receive raises in the caller
    within the timeout, the leg is recorded as an error on both ranks, the later
    collective leg is skipped on both (no mismatched collective), the local leg
    still runs, and rank 0 prints the one line with the headline value."""
    import socket
    import time
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    t0 = time.time()
    procs = [subprocess.Popen([sys.executable, "-c", _LEGS_WORKER], cwd=ROOT, stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True,
                              env=_env(ROOT=ROOT, MODE=mode, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                                       MASTER_PORT=str(port)))
             for r in range(2)]
    outs = [p.communicate(timeout=180) for p in procs]
    assert time.time() - t0 < 120
    status = {}
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
        for ln in o.splitlines():
            if ln.startswith("STATUS"):
                _, r, js = ln.split(" ", 2)
                status[int(r)] = json.loads(js)
    lines = [x for x in outs[0][0].splitlines() if x.startswith("{")]
    assert len(lines) == 1 and not any(x.startswith("{") for x in outs[1][0].splitlines())
    d = json.loads(lines[0])
    assert d["value"] == 123.0 and d["ag"] == [0.0, 1.0] and d["p2p"] is None and d["local"] == 7, d
    assert d["elapsed"] < 30, d
    for r in (0, 1):
        s = status[r]
        assert s["ag"]["ok"] and s["local"]["ok"], (r, s)
        assert "error" in s["p2p"], (r, s)
        assert "skipped" in s["after"], (r, s)
    assert "injected" in status[1]["p2p"]["error"]
    assert d["legs"] == status[0]


_WATCHDOG_WORKER = r"""
import os, sys, time
sys.path.insert(0, os.environ["ROOT"])
import bench
rep = bench.Report(0)
rep.out = {"value": 5.0}
legs = bench.Legs(rep, False, deadline_s=1.5)
rep.out["legs"] = legs.status
rep.out["fine"] = legs.run("fine", lambda: 1, collective=False)
legs.run("stuck", lambda: time.sleep(60), collective=False)
print("NOT REACHED", flush=True)
"""


def test_legs_watchdog_prints_the_line():
    """A leg stuck past its deadline (a hang no collective timeout reaches): the
    watchdog prints the line with the headline, the finished legs and the stuck
    leg's error, and the process exits 0 without waiting for the leg."""
    import time
    t0 = time.time()
    r = subprocess.run([sys.executable, "-c", _WATCHDOG_WORKER], cwd=ROOT, env=_env(ROOT=ROOT),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    assert time.time() - t0 < 40
    lines = [x for x in r.stdout.splitlines() if x.strip()]
    assert len(lines) == 1 and "NOT REACHED" not in r.stdout, r.stdout
    d = json.loads(lines[0])
    assert d["value"] == 5.0 and d["fine"] == 1 and d["legs"]["fine"]["ok"] is True, d
    assert "deadline" in d["legs"]["stuck"]["error"], d


def test_merge_methods_and_fault_injection():
    """bench.merge_methods joins a gather leg's all-gather and p2p halves (which run as separate,
    fail-soft legs): flags hold over the methods that ran, a missing half carries its leg status,
    and the gathered tensors are compared when both ran.  inject_p2p_fault touches only the last
    rank's p2p leg."""
    import types
    import torch
    sys.path.insert(0, ROOT)
    import bench
    full = torch.arange(12, dtype=torch.int16).reshape(3, 4)
    a = {"methods": {"all_gather": {"gathered_equals_unsharded": True}}, "gathered_equals_unsharded": True,
         "own_slice_intact": True, "methods_gather_the_same": True, "_full": full}
    p = {"methods": {"p2p": {"gathered_equals_unsharded": False}}, "gathered_equals_unsharded": False,
         "own_slice_intact": True, "methods_gather_the_same": True, "_full": full.clone()}
    m = bench.merge_methods(a, p, "p2p", None)
    assert set(m["methods"]) == {"all_gather", "p2p"} and "_full" not in m
    assert m["gathered_equals_unsharded"] is False and m["own_slice_intact"] is True
    assert m["methods_gather_the_same"] is True
    p2 = dict(p, _full=full + 1)
    assert bench.merge_methods(a, p2, "p2p", None)["methods_gather_the_same"] is False
    st = {"error": "TimeoutError: gloo recv"}
    m = bench.merge_methods(a, None, "p2p", st)
    assert m["methods"]["p2p"] == st and m["gathered_equals_unsharded"] is True and m["methods_gather_the_same"] is None
    assert bench.merge_methods(None, None, "p2p", st) is None
    assert bench.merge_methods(None, p, "p2p", None)["methods"] == p["methods"]
    args = types.SimpleNamespace(gather_fault="p2p-raise", dist_timeout=1.0)
    bench.inject_p2p_fault(args, 4, 2, "p2p")  # not the last rank
    bench.inject_p2p_fault(args, 4, 3, "all_gather")  # not the p2p leg
    with pytest.raises(RuntimeError, match="injected"):
        bench.inject_p2p_fault(args, 4, 3, "p2p")
    bench.inject_p2p_fault(types.SimpleNamespace(gather_fault="offset", dist_timeout=1.0), 4, 3, "p2p")
