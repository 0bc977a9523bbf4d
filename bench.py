#!/usr/bin/env python3
"""bench.py -- MI355X throughput of the 8x8 DCT + quantization hot path.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--frames F] [--quality Q]
                    [--adaptive 0|1] [--kind uniform|smooth|const|extreme]

Metric (BASELINE.json): 8x8 macroblocks/s (DCT+quant) and % of HBM roofline.
Workload: a stream of 4K 4:2:0 frames (BASELINE configs[2] planes: Y 3840x2160 +
Cb/Cr 1920x1080 = 194,400 blocks per frame), F frames per GPU per step, resident
in HBM; one step = dctq_forward_quant_planes over every block of the batch (ONE
launch: plane 0 = the F luma frames, plane 1 = the 2F chroma frames; --per-plane
times the two-launch form), int16 coefficients bit-exact with the reference.  N>1: one process per GPU (torch.distributed),
each rank its own F frames (weak scaling, no data-path collective); value =
all blocks / max-over-ranks wall time.  A separately reported leg
("round_trip", BASELINE configs[4]) runs forward DCT+quant then dequant+IDCT
over the same frames in ONE fused launch (dctq_round_trip_planes) and reports
end-to-end blocks/s (the unfused two-kernel pair timed beside it) and PSNR.
Another ("encode") runs the encoder (forward + zigzag run-length
symbols) over the frames, and at N>1 the all-gather of the symbol streams.  At N>1 a
second, separately reported leg ("gather") times forward DCT+quant of the luma frames followed by the RCCL
all-gather of every rank's int16 coefficient planes (BASELINE configs[3],
SURVEY 8(e)(ii)) -- strong scaling: --total-frames 4K luma frames (64) split
over the ranks, the kernel-only aggregate rate and the rate including the
xGMI exchange reported apart; and "band" splits ONE 4K 4:2:0 frame across the
ranks in block-row bands and all-gathers its coefficient planes (latency per
frame).

Also reported: the dominant kernel's roofline (algorithmic 192 B/block over the
HIP-event-timed launch durations), the memory ceilings of its traffic measured
on the same box (roofline.movement_ceiling: its own movement and the best flat
1:2 stream; roofline.hw_ceilings), and the reference's own CPU path
(oracle/_ref/libref.so and libref_O0.so: src/dct.c + src/quantization.c
compiled from /root/reference with -O2 and with the Justfile's -g) timed on
this host's cores in the same run, all cores and one thread.  That CPU leg
(cpu_leg, rank 0) is also where the oracle checks this run's GPU outputs (one
chroma plane's coefficients and Huffman sizes): oracle/ is a checker here,
never the thing measured.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import dct_amd  # noqa: E402

HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md)
BYTES_PER_BLOCK = 64 + 128  # u8 in + int16 out
Y_W, Y_H, C_W, C_H = 3840, 2160, 1920, 1080


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--frames", type=int, default=64, help="4K 4:2:0 frames per GPU per step")
    ap.add_argument("--quality", type=int, default=50)
    ap.add_argument("--adaptive", type=int, default=0)
    ap.add_argument("--kind", default="uniform")
    ap.add_argument("--seed", type=int, default=12345)
    ap.add_argument("--cpu-seconds", type=float, default=20.0,
                    help="CPU-baseline sample budget (wall s, over its four builds x thread counts)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic.json"))
    ap.add_argument("--gather-steps", type=int, default=3, help="N>1: timed forward+all-gather steps (0 = skip)")
    ap.add_argument("--total-frames", type=int, default=64,
                    help="N>1 gather leg (BASELINE configs[3]): 4K luma frames in total, split over the ranks")
    ap.add_argument("--gather-fault", default="none", choices=["none", "offset", "p2p-raise", "p2p-stall"],
                    help="tests only: 'offset' makes every rank transform the frames one past its own slice (a "
                         "wrong shard offset shared by both gather shapes), so the gather leg's "
                         "gathered_equals_unsharded must read false; 'p2p-raise' / 'p2p-stall' make the last rank "
                         "raise before posting its direct pushes / sleep past --dist-timeout first, so its peers' "
                         "p2p gather times out (the line must still carry the headline and the leg's error)")
    ap.add_argument("--dist-timeout", type=float, default=90.0,
                    help="N>1: process-group timeout in seconds (a collective still waiting on a peer after it "
                         "raises in the caller; the optional legs are fail-soft, class Legs)")
    ap.add_argument("--leg-deadline", type=float, default=0.0,
                    help="watchdog bound on each optional leg in seconds (0 = 2 x --dist-timeout + 60)")
    ap.add_argument("--encode-steps", type=int, default=10,
                    help="timed steps of the encoder leg (forward + zigzag/RLE symbols; at N>1 plus the "
                         "symbol-stream all-gather); 0 = skip")
    ap.add_argument("--round-trip-steps", type=int, default=10,
                    help="timed steps of the config-5 round trip leg (forward+inverse, PSNR); 0 = skip")
    ap.add_argument("--ceiling-rounds", type=int, default=10,
                    help="interleaved forward / no-arithmetic movement launches for roofline.movement_ceiling (0 = skip)")
    ap.add_argument("--prewarm-ms", type=float, default=250.0,
                    help="untimed GPU pre-warm before the warmup steps: the step runs back to back for this long so "
                         "the timed steps see steady-state clocks (an idle MI355X sits at ~100 MHz sclk and needs "
                         "~25 ms of load to ramp: profiles/r02/clock_ramp.md)")
    ap.add_argument("--per-plane", action="store_true",
                    help="two launches per step (luma, then chroma) instead of one multi-plane launch")
    ap.add_argument("--dist-legs", action="store_true",
                    help="at one process: form a one-rank process group (--backend) and run the N>1 legs anyway "
                         "(gather, band, symbol-stream gather): the RCCL code path on a single GPU")
    ap.add_argument("--backend", default="nccl", help="N>1 process group (nccl = RCCL; gloo only to rehearse "
                                                      "several ranks on one GPU)")
    ap.add_argument("--launch-check", action="store_true",
                    help="rank plumbing only, no GPU: every rank joins a gloo group and rank 0 prints the world it "
                         "formed (tests/test_bench_launch.py)")
    return ap.parse_args()


class _StdoutToStderr:
    """fd 1 -> fd 2 for the duration: gloo's C++ rendezvous prints "[Gloo] Rank r is connected
    ..." to stdout, and rank 0's stdout must carry the one JSON line only."""

    def __enter__(self):
        sys.stdout.flush()
        self._saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self._saved, 1)
        os.close(self._saved)
        return False


def trace(msg: str) -> None:
    """One progress line on stderr (DCTQ_BENCH_TRACE=1): which leg a failure came from."""
    if os.environ.get("DCTQ_BENCH_TRACE") == "1":
        print(f"[bench rank {os.environ.get('RANK', '0')}] {msg}", file=sys.stderr, flush=True)


class Report:
    """Rank 0's one JSON line, filled in as the legs finish and printed exactly
    once: by main() at the end, or by the leg watchdog (Legs) when a leg outlives
    its deadline -- then with the headline, every leg that finished and the
    stuck leg's error.  The headline is measured before any optional leg runs,
    so no later leg can lose it."""

    def __init__(self, rank: int):
        import threading
        self.rank = rank
        self.out = None
        self._lock = threading.Lock()
        self._printed = False

    def emit(self) -> None:
        with self._lock:
            if self._printed or self.rank != 0 or self.out is None:
                return
            self._printed = True
            for _ in range(3):  # the watchdog may serialise while the main thread adds a key
                try:
                    line = json.dumps(self.out, default=str)
                    break
                except RuntimeError:
                    time.sleep(0.01)
            else:
                line = json.dumps(dict(self.out), default=str)
            print(line, flush=True)


class Legs:
    """Fail-soft runner of bench.py's optional legs (everything after the headline).

    run(name, fn, collective) calls fn() and records legs[name] = {"ok": true,
    "seconds": ...} or {"error": "..."}; an exception is reported, never raised.
    A collective leg that fails leaves this rank's process group untrusted (a peer
    may still be inside the collective it abandoned), so every LATER collective
    leg on this rank is skipped ({"skipped": ...}) rather than risk a mismatched
    or hanging collective; a peer that is left waiting for this rank then times
    out in its own collective (the process group's timeout: gloo's per-operation
    timeout; for RCCL, TORCH_NCCL_BLOCKING_WAIT=1, which main() sets, makes the
    waiting call raise in the caller at the timeout instead of a watchdog thread
    tearing the process down) and skips its later legs the same way.

    A watchdog thread bounds every leg by `deadline_s` (a hang inside a kernel or
    a collective that no timeout reaches): past it, rank 0 prints the Report with
    that leg's error and every process exits with status 0 (os._exit: no exec,
    nothing waits on the stuck stream)."""

    def __init__(self, report: Report, dist_on: bool, deadline_s: float):
        import threading
        self.report = report
        self.dist_on = dist_on
        self.deadline_s = deadline_s
        self.status = {}
        self.poisoned = None
        self._armed = None
        self._cv = threading.Condition()
        threading.Thread(target=self._watch, name="bench-leg-watchdog", daemon=True).start()

    def _watch(self):
        with self._cv:
            while True:
                if self._armed is None:
                    self._cv.wait()
                    continue
                name, t_end = self._armed
                left = t_end - time.monotonic()
                if left <= 0:
                    break
                self._cv.wait(left)
        self.status[name] = {"error": f"exceeded its {self.deadline_s:.0f} s deadline (leg watchdog): "
                                      "the line was printed and the process exited"}
        print(f"bench.py: leg {name} exceeded {self.deadline_s:.0f} s; printing the line and exiting",
              file=sys.stderr, flush=True)
        self.report.emit()
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)

    def run(self, name: str, fn, collective: bool = True):
        import traceback
        if collective and self.dist_on and self.poisoned:
            self.status[name] = {"skipped": f"after leg {self.poisoned} failed on this rank (its process group "
                                            "can no longer be trusted)"}
            trace(f"leg {name}: skipped")
            return None
        trace(f"leg {name}")
        with self._cv:
            self._armed = (name, time.monotonic() + self.deadline_s)
            self._cv.notify()
        t0 = time.perf_counter()
        try:
            r = fn()
            self.status[name] = {"ok": True, "seconds": round(time.perf_counter() - t0, 3)}
            return r
        except Exception as e:  # noqa: BLE001 -- recorded in the line, never raised
            self.status[name] = {"error": f"{type(e).__name__}: {e}"[:800],
                                 "seconds": round(time.perf_counter() - t0, 3)}
            print(f"bench.py: leg {name} failed on rank {self.report.rank}:", file=sys.stderr)
            traceback.print_exc(file=sys.stderr)
            if collective and self.dist_on:
                self.poisoned = name
            return None
        finally:
            with self._cv:
                self._armed = None
                self._cv.notify()


def spawn_ranks(n: int) -> int:
    """`--gpus N` (N > 1) with no launcher around this process: start N copies of
    this command as child processes, one per GPU, with the environment
    torch.distributed.run would give them (RANK, LOCAL_RANK, WORLD_SIZE,
    LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, a free MASTER_PORT), wait for all of
    them, and return the exit status.  This parent never touches the GPU (no HIP
    call, not even a device count) and never exec()s: the children are ordinary
    subprocesses.  Rank 0 inherits stdout, so its one JSON line is this command's
    output; if any rank fails, the others are stopped (by PID) and the status is
    the failing rank's."""
    import signal
    import socket
    import subprocess
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    def die_with_parent():  # in the child, before it runs anything: SIGTERM if this launcher dies
        import ctypes
        ctypes.CDLL(None, use_errno=True).prctl(1, signal.SIGTERM)  # PR_SET_PDEATHSIG

    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else sys.stderr, preexec_fn=die_with_parent))

    def forward(signum, _frame):  # a time limit on this launcher reaches the ranks too
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        sys.exit(128 + signum)

    signal.signal(signal.SIGTERM, forward)
    signal.signal(signal.SIGINT, forward)
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                print(f"bench.py: rank {procs.index(p)} exited with {c}; stopping the other ranks", file=sys.stderr)
                for q in live:
                    q.send_signal(signal.SIGTERM)
        if live:
            time.sleep(0.05)
    return rc


def launch_check(args) -> None:
    """--launch-check: each rank joins a gloo group over the env rendezvous and
    contributes its rank; rank 0 prints the world it saw.  No GPU."""
    with _StdoutToStderr():
        dist.init_process_group("gloo")
    t = torch.tensor([dist.get_rank()], dtype=torch.int64)
    dist.all_reduce(t)
    if dist.get_rank() == 0:
        print(json.dumps({"n_gpus": args.gpus, "world_size": dist.get_world_size(), "rank_sum": int(t.item()),
                          "backend": dist.get_backend()}))
    dist.destroy_process_group()


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def gpu_identity():
    """The box's GPU as rocm-smi reports it (serial, HBM vendor, memory/compute partition):
    boxes of this pool differ by up to ~15 % on the same bytes (HISTORY.md 3.1b), and the
    bench's own ceilings are the normaliser; this says which box a line came from."""
    import re
    import shutil
    import subprocess
    if "rocprof" in os.environ.get("LD_PRELOAD", ""):
        # under rocprofv3 every child process gets the profiler preloaded (with --pmc it
        # initialises the GPU), and rocm-smi's `#!/usr/bin/env python3` would then exec
        # after GPU initialisation: skip the query in profiling runs
        return None
    smi = shutil.which("rocm-smi") or "/opt/rocm/bin/rocm-smi"
    try:
        with open(smi, "rb") as f:
            first = f.readline()
    except OSError:
        return None
    script = first.startswith(b"#!") and b"python" in first  # run it with this interpreter: no env hop
    cmd = ([sys.executable, smi] if script else [smi]) + ["--showserial", "--showmemvendor",
                                                         "--showmemorypartition", "--showcomputepartition"]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=30)
    except (OSError, subprocess.SubprocessError):
        return None
    keys = {"Serial Number": "serial", "GPU memory vendor": "hbm_vendor", "Memory Partition": "memory_partition",
            "Compute Partition": "compute_partition"}
    ident = {}
    for line in r.stdout.splitlines():
        m = re.match(r"GPU\[0\]\s*:\s*([^:]+?):\s*(\S+)", line)
        if m and m.group(1).strip() in keys:
            ident[keys[m.group(1).strip()]] = m.group(2)
    return ident or None


def cpu_share():
    """CPUs this process may use: the cgroup CPU quota if one is set, else the
    scheduler affinity mask; capped by OMP_NUM_THREADS when the environment
    declares a smaller share (the GPU box's harness sets it to the per-GPU share
    of the host's cores).  Returns (threads, how)."""
    aff = len(os.sched_getaffinity(0))
    n, how = aff, f"affinity mask ({aff} CPUs)"
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            q = max(1, int(int(quota) / int(period)))
            if q < n:
                n, how = q, f"cgroup cpu.max quota ({quota}/{period})"
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and 0 < int(omp) < n:
        n, how = int(omp), f"OMP_NUM_THREADS={omp} (this host's CPU share per GPU; affinity {aff})"
    return n, how


def cpu_baseline(args):
    """The reference CPU path on this host, a bounded sample of the same workload
    (BASELINE.md "CPU-baseline plan"): the reference's own per-block pipeline over
    4K 4:2:0 frames, pthreads over block rows with a shared read-only ctx, built
    with -O2 and with the Justfile's flags (-g, i.e. -O0), on every CPU of this
    process's share (cpu_share) and on one thread.  `value` = -O2 on the share."""
    import numpy as np
    import oracle as O
    cores, share = cpu_share()
    kind = "reference" if O.ref_available() else "port"
    frames = [O.synth_plane(args.seed, O.KINDS[args.kind], Y_W, Y_H),
              O.synth_plane(args.seed + 1, O.KINDS[args.kind], C_W, C_H),
              O.synth_plane(args.seed + 2, O.KINDS[args.kind], C_W, C_H)]
    outs = [np.zeros(((f.shape[0] // 8) * (f.shape[1] // 8), 64), np.int16) for f in frames]

    def run(build, threads, budget):
        nblk, nfr, t0 = 0, 0, time.perf_counter()
        while True:
            for f, o in zip(frames, outs):
                if kind == "reference":
                    O.ref(build).ref_forward_plane(f.ravel(), f.shape[1], f.shape[0], args.quality, args.adaptive,
                                                   o.ravel(), threads, 0)
                else:
                    o[:] = O.forward_plane(f, args.quality, args.adaptive, threads)
                nblk += o.shape[0]
            nfr += 1
            el = time.perf_counter() - t0
            if el >= budget:
                return {"value": nblk / el, "threads": threads, "frames": nfr, "blocks": nblk, "seconds": el}

    budget = args.cpu_seconds
    legs = {"O2_all_cores": run("O2", cores, 0.4 * budget), "O2_one_thread": run("O2", 1, 0.2 * budget)}
    if kind == "reference":
        legs.update({"O0_all_cores": run("O0", cores, 0.2 * budget), "O0_one_thread": run("O0", 1, 0.2 * budget)})
    head = legs["O2_all_cores"]
    return {"value": head["value"], "unit": "macroblocks/s", "cores": cores, "kind": kind,
            "nproc": cores, "cpu_share": share, "machine_cpus": os.cpu_count(), "cpu_model": cpu_model(),
            "sample": f"{head['frames']} 4K 4:2:0 frame(s) ({head['blocks']} blocks, {args.kind}, q{args.quality}, "
                      f"adaptive={args.adaptive}) through the reference's create_block_from_pixels -> dct_forward -> "
                      f"calculate_block_variance -> quantize per block (oracle/_ref/libref.so, -O2), {cores} pthreads "
                      f"over block rows ({share}), {head['seconds']:.1f} s",
            "builds": {k: {"blocks_per_s": v["value"], "threads": v["threads"], "blocks": v["blocks"],
                           "seconds": round(v["seconds"], 2)} for k, v in legs.items()},
            "flags": {"O2": "-Wall -Wextra -Werror -pedantic -std=c99 -O2 -fPIC (oracle/Makefile REFFLAGS)",
                      "O0": "-Wall -Wextra -Werror -pedantic -std=c99 -g -fPIC (Justfile:8 CFLAGS)"}}


def cpu_leg(args, world, fwd_check, huf_check, rt_check=None):
    """The CPU leg (rank 0): the reference's own CPU path timed on this host
    (cpu_baseline, N=1 only), and the oracle as CHECKER of this run's GPU
    outputs -- one chroma plane's coefficients and its per-block Huffman sizes.
    The only part of bench.py that touches oracle/ (besides small_frame's
    reference timing)."""
    import numpy as np
    import oracle as O
    parity = {}
    try:
        if fwd_check is not None:
            px, got = fwd_check
            parity["forward"] = bool(np.array_equal(got, O.forward_plane(px, args.quality, args.adaptive, 8)))
        if huf_check is not None:
            c, b = huf_check
            parity["huffman"] = bool(np.array_equal(b.view(np.uint32), O.huffman_bits_plane(c)))
        if rt_check is not None:
            parity["round_trip"] = round_trip_parity(args, rt_check)
    except Exception as e:  # noqa: BLE001 -- report, do not hide
        parity["error"] = str(e)
    cpu = cpu_baseline(args) if world == 1 else None
    return cpu, parity


def round_trip_parity(args, ck):
    """The fused round trip's output for chroma frame 0 against the oracle:
    coefficients bit-exact (forward_plane), recon within 1e-4 of
    dct_inverse(dequantize()) + 128 (inverse_plane; src/quantization.c:133-151,
    src/dct.c:80-105), and luma frame 0's PSNR equal to the oracle pipeline's
    (tests/test_entropy.c:376-393 formula, recon clamped to [0, 255])."""
    import math
    import numpy as np
    import oracle as O
    q, ad = args.quality, args.adaptive
    want_c = O.forward_plane(ck["px"], q, ad, 8)
    var = O.plane_variance(ck["px"]) if ad else None
    want_r = O.inverse_plane(want_c, q, ad, var) + 128.0
    err = float(np.abs(ck["recon"].astype(np.float64) - want_r).max())
    y = ck["luma0"]
    h, w = y.shape
    yc = O.forward_plane(y, q, ad, 8)
    yr = O.inverse_plane(yc, q, ad, O.plane_variance(y) if ad else None) + 128.0
    blocks = y.reshape(h // 8, 8, w // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64).astype(np.float64)
    mse = float(((blocks - np.clip(yr, 0, 255)) ** 2).mean())
    psnr = float("inf") if mse == 0 else 10.0 * math.log10(255.0 * 255.0 / mse)
    return {"coef_bit_exact": bool(np.array_equal(ck["coef"], want_c)), "recon_max_abs_err": err,
            "recon_within_1e-4": err <= 1e-4, "psnr_oracle_db": psnr, "psnr_gpu_db": ck["psnr"],
            "psnr_abs_diff": abs(psnr - ck["psnr"]), "blocks": int(want_c.shape[0])}


def inject_p2p_fault(args, world, rank, method):
    """--gather-fault p2p-raise / p2p-stall: the last rank fails its direct-push
    gather before posting anything (p2p-stall first sleeps past the process
    group's timeout), so its peers' grouped send/recv wait on it and time out."""
    if method != "p2p" or rank != world - 1 or not args.gather_fault.startswith("p2p-"):
        return
    if args.gather_fault == "p2p-stall":
        time.sleep(args.dist_timeout + 10.0)
    raise RuntimeError(f"injected fault (--gather-fault {args.gather_fault}) on rank {rank}")


def merge_methods(first, second, second_method, status):
    """One gather/band result from its per-method legs: `first` (the all-gather
    leg's dict, or None if it failed) and `second` (the p2p leg's, or None with
    the reason in `status`).  The summary flags hold over the methods that ran."""
    if first is None and second is None:
        return None
    base = dict(first if first is not None else second)
    full0 = base.pop("_full", None)
    methods = dict(base["methods"])
    if second is not None and first is not None:
        methods.update(second["methods"])
        full1 = second.get("_full")
        if full0 is not None and full1 is not None:
            if "methods_gather_the_same" in base:
                base["methods_gather_the_same"] = bool(torch.equal(full0, full1))
        for k in ("gathered_equals_unsharded", "own_slice_intact"):
            if k in base and k in second:
                base[k] = bool(base[k] and second[k])
    elif first is not None:
        methods[second_method] = status or {"error": "did not run"}
        if "methods_gather_the_same" in base:
            base["methods_gather_the_same"] = None
    base["methods"] = methods
    return base


def band_leg(args, plan, luma, chroma, world, dev, methods, reps=20):
    """N>1, the north_star's literal split: ONE 4K 4:2:0 frame (its Y, Cb and Cr
    planes) partitioned across the ranks in block-row bands
    (dct_amd.shard.band_shard), forward DCT+quant of every band in one
    multi-plane launch, then the coefficient planes all-gathered so every rank
    holds the whole frame's coefficients (one collective for the three planes,
    shard.gather_planes; ragged bands padded).  Latency-bound (194 400 blocks per frame); max-over-ranks wall
    time per frame, and a check of the gathered planes against an unsharded
    forward on this rank.  `methods`: the gather shapes this call runs (main()
    runs the all-gather leg first and the direct pushes as a separate, last leg)."""
    from dct_amd import shard
    # the same frame on every rank (each uses only its band of it)
    y = dct_amd.synth(args.seed + 777, args.kind, luma.shape[-1], luma.shape[-2], 1, device=dev)
    c = dct_amd.synth(args.seed + 778, args.kind, chroma.shape[-1], chroma.shape[-2], 2, device=dev)
    planes = [y[0], c[0], c[1]]
    bands, outs, counts = [], [], []
    for p in planes:
        band, (_, rows) = shard.band_shard(p, world, dist.get_rank())
        bw = p.shape[-1] // 8
        bands.append(band)
        outs.append(torch.empty((rows * bw, 64), dtype=torch.int16, device=dev))
        counts.append([(hi - lo) * bw for lo, hi in (shard.split(p.shape[-2] // 8, world, r) for r in range(world))])

    def timed(fn):
        r = fn()
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            r = fn()
        torch.cuda.synchronize()
        return shard.max_over_ranks(time.perf_counter() - t0, dev), r

    want = plan.forward_quant_planes(planes)
    nblk = sum(w.shape[0] for w in want)
    rank = dist.get_rank()
    recv = sum(sum(c) - c[rank] for c in counts) * 128
    by = {}
    for m in methods:  # SURVEY 8(e)'s two shapes: the all-gather collective, direct peer pushes
        inject_p2p_fault(args, world, rank, m)

        def once():
            plan.forward_quant_planes(bands, outs=outs)
            return shard.gather_planes(outs, counts, method=m)  # the three planes in one collective / one group
        el, full = timed(once)
        el_g, _ = timed(lambda: shard.gather_planes(outs, counts, method=m))  # the exchange alone
        by[m] = {"op": gather_op_name(m), "us_per_frame": el / reps * 1e6, "blocks_per_s": nblk * reps / el,
                 "gathered_equals_unsharded": all(bool(torch.equal(f, w)) for f, w in zip(full, want)),
                 "xgmi": shard.xgmi_report(recv, el_g / reps, world)}
    first = by[methods[0]]
    return {"op": f"one 4K 4:2:0 frame in block-row bands over {world} ranks: forward_quant_planes(bands) + "
                  f"{first['op']} of the Y/Cb/Cr coefficient planes", "frames": reps,
            "us_per_frame": first["us_per_frame"], "blocks_per_s": first["blocks_per_s"],
            "gathered_equals_unsharded": all(v["gathered_equals_unsharded"] for v in by.values()),
            "xgmi": first["xgmi"], "methods": by}


def gather_op_name(method):
    """What a gather method runs on this process group's backend (bench JSON 'op' strings)."""
    nccl = dist.get_backend() == "nccl"
    if method == "p2p":
        # first multi-rank RCCL run of this shape: its own gathered_equals_unsharded is the check
        return ("RCCL grouped ncclSend/ncclRecv direct pushes (batch_isend_irecv; unverified on hardware before "
                "this run, see gathered_equals_unsharded)" if nccl
                else f"{dist.get_backend()} isend/irecv direct pushes (batch_isend_irecv)")
    return "RCCL all_gather_into_tensor" if nccl else f"{dist.get_backend()} all_gather"


def gather_leg(args, plan, world, rank, dev, methods):
    """BASELINE configs[3], strong scaling: --total-frames 4K luma frames (64)
    split over the ranks (shard.split: 8 per GPU at N=8), forward DCT+quant of
    each rank's frames, then the RCCL all-gather of every rank's int16
    coefficient planes onto every rank (shard.strong_gather_leg).  Reports the
    kernel-only aggregate (what the GPUs transform per second together) and the
    end-to-end rate with the exchange, apart: SURVEY 8(e) prices the gather at
    25-170x the compute, so it is bound by xGMI, not by the kernel.  `methods`:
    the gather shapes this call runs (main() runs the all-gather first, the
    direct pushes as the last leg); the gathered tensor rides along as "_full"
    so merge_methods can compare the shapes."""
    from dct_amd import shard
    for m in methods:
        inject_p2p_fault(args, world, rank, m)
    lo, hi = shard.split(args.total_frames, world, rank)
    per = (Y_W // 8) * (Y_H // 8)
    # frame f of synth(seed, n) is made from seed + f, so seeding by the global index of the
    # shard's first frame makes the shards tile the unsharded stack exactly
    first = (lo + 1) % args.total_frames if args.gather_fault == "offset" else lo
    frames = dct_amd.synth(args.seed + 200000 + first, args.kind, Y_W, Y_H, max(hi - lo, 1), device=dev)[:hi - lo]
    out = torch.empty(((hi - lo) * per, 64), dtype=torch.int16, device=dev)
    counts = [(b - a) * per for a, b in (shard.split(args.total_frames, world, r) for r in range(world))]

    def forward(fr):
        if fr.shape[0]:
            plan.forward_quant(fr, out=out)
        return out

    def unsharded(chunk=8):
        """The unsharded forward of all --total-frames frames, recomputed on this rank
        chunk by chunk (8 frames at a time): what every rank must hold after a gather."""
        buf = torch.empty((chunk, Y_H, Y_W), dtype=torch.uint8, device=dev)
        for g0 in range(0, args.total_frames, chunk):
            n = min(chunk, args.total_frames - g0)
            fr = dct_amd.synth(args.seed + 200000 + g0, args.kind, Y_W, Y_H, n, device=dev, out=buf[:n])
            yield g0 * per, plan.forward_quant(fr)

    r = shard.strong_gather_leg(forward, frames, counts, args.gather_steps, dev, torch.cuda.synchronize,
                                methods=methods, unsharded=unsharded)
    local = r["local"]
    off = sum(counts[:rank])
    n = r["blocks_per_step"] * r["steps"]
    recv = (sum(counts) - counts[rank]) * 128
    by = {m: {"op": gather_op_name(m), "blocks_per_s": n / v["end_to_end_s"],
              "ms_per_step": v["end_to_end_s"] / r["steps"] * 1e3,
              "own_slice_intact": bool(torch.equal(v["full"][off:off + counts[rank]], local)),
              "gathered_equals_unsharded": v["gathered_equals_unsharded"],
              "xgmi": shard.xgmi_report(recv, v["gather_s"] / r["steps"], world)}
          for m, v in r["by_method"].items()}
    full0 = r["full"]
    same = all(bool(torch.equal(v["full"], full0)) for v in r["by_method"].values())
    # every rank checked its own copy: the leg passes only if all of them hold the unsharded result
    ok = torch.tensor([int(all(v["gathered_equals_unsharded"] for v in by.values()))], device=dev)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    first_m = by[methods[0]]
    return {"op": f"{args.total_frames} 4K luma frames split over {world} ranks: forward_quant + {first_m['op']} of "
                  "the int16 coefficient planes (BASELINE configs[3])", "scaling": "strong", "world_size": world,
            "frames_total": args.total_frames, "frames_this_rank": hi - lo, "steps": r["steps"],
            "kernel_blocks_per_s": n / r["kernel_s"], "kernel_ms_per_step": r["kernel_s"] / r["steps"] * 1e3,
            "blocks_per_s": first_m["blocks_per_s"], "ms_per_step": first_m["ms_per_step"],
            "bytes_received_per_rank": recv, "own_slice_intact": all(v["own_slice_intact"] for v in by.values()),
            "methods_gather_the_same": same, "gathered_equals_unsharded": bool(ok.item()),
            "fault_injected": args.gather_fault, "xgmi": first_m["xgmi"], "methods": by, "_full": full0}


def small_frame_leg(args, plan, dev):
    """BASELINE configs[1]: one 512x512 grayscale frame (4 096 blocks, 256 KiB in,
    512 KiB out: cache-resident, so launch-bound -- not an HBM-roofline figure),
    200 back-to-back dctq_forward_quant launches, next to the reference's CPU
    path on the same frame (oracle/_ref, every core of this process, rank 0 only)."""
    import numpy as np
    import oracle as O
    px = dct_amd.synth(args.seed + 7, args.kind, 512, 512, device=dev)
    out = torch.empty((4096, 64), dtype=torch.int16, device=dev)
    n = 200
    for _ in range(10):
        plan.forward_quant(px, out=out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        plan.forward_quant(px, out=out)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    res = {"frame": "512x512 u8 (4096 blocks)", "launches": n, "us_per_frame": el / n * 1e6,
           "blocks_per_s": 4096 * n / el}
    # the same launches captured once into a HIP graph and replayed (the host's
    # per-call cost -- ctypes, argument checks, hipLaunchKernel -- paid at capture)
    try:
        per_graph, replays = 100, 4
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            plan.forward_quant(px, out=out)
        torch.cuda.current_stream().wait_stream(side)
        with torch.cuda.graph(g):
            for _ in range(per_graph):
                plan.forward_quant(px, out=out)
        g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(replays):
            g.replay()
        torch.cuda.synchronize()
        elg = time.perf_counter() - t0
        res.update({"graph_launches": per_graph * replays, "graph_us_per_frame": elg / (per_graph * replays) * 1e6,
                    "graph_blocks_per_s": 4096 * per_graph * replays / elg})
    except Exception as e:  # noqa: BLE001 -- report, do not hide
        res["graph_error"] = str(e)
    host = px[0].cpu().numpy()
    got = out.cpu().numpy()
    if O.ref_available():
        ref = np.zeros((4096, 64), np.int16)
        threads = cpu_share()[0]
        reps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < 1.0:
            O.ref().ref_forward_plane(np.ascontiguousarray(host).ravel(), 512, 512, args.quality, args.adaptive,
                                      ref.ravel(), threads, 0)
            reps += 1
        res.update({"cpu_reference_blocks_per_s": 4096 * reps / (time.perf_counter() - t0), "cpu_threads": threads,
                    "bit_exact_vs_reference": bool(np.array_equal(got, ref))})
    return res


def legacy_leg(args, dev, threads=(1, 8)):
    """The reference's per-block API served by libdct_amd.so (include/dct.h,
    include/quantization.h): host/block_pipeline_mt.c runs the reference's forward
    loop (create_block_from_pixels -> dct_forward -> calculate_block_variance ->
    quantize, tests/test_entropy.c:300-316) over every block of one 256x128 plane
    from 1 and from 8 host threads sharing one context (legacy.hip: a lane per
    thread, no lock after a thread's first call), a child process of its own.
    Latency-bound by design (one block per call, as in the reference); reported
    next to the reference's one-thread CPU rate as a stated baseline, not a target.
    Self-checked: the 8-thread output equals the 1-thread output."""
    import subprocess
    import tempfile
    exe = os.path.join(ROOT, "host", "block_pipeline_mt")
    if not os.path.exists(exe):
        raise RuntimeError(f"{exe} is not built (make -C host)")
    w, h = 256, 128
    px = dct_amd.synth(args.seed + 31, args.kind, w, h, device=dev)[0].cpu().numpy()
    res = {"op": "reference per-block forward loop through the legacy C API (host/block_pipeline_mt.c), "
                 f"{w}x{h} plane, q{args.quality} adaptive={args.adaptive}", "blocks": (w // 8) * (h // 8)}
    with tempfile.TemporaryDirectory() as tmp:
        pf = os.path.join(tmp, "px.u8")
        px.tofile(pf)
        outs = {}
        for t in threads:
            of = os.path.join(tmp, f"out{t}.bin")
            r = subprocess.run([exe, pf, str(w), str(h), str(args.quality), str(args.adaptive), str(t), "4", of,
                                "forward"], capture_output=True, text=True, timeout=120)
            if r.returncode != 0:
                raise RuntimeError(f"block_pipeline_mt {t} threads: rc {r.returncode}: {r.stderr[-500:]}")
            kv = dict(ln.split(":", 1) for ln in r.stdout.strip().splitlines())
            outs[t] = open(of, "rb").read()
            res[f"threads_{t}"] = {"blocks_per_s": float(kv["pipelines_per_s"]), "calls_per_s": float(kv["calls_per_s"]),
                                   "rand_undisturbed": kv["rand_ok"] == "1"}
    res["threads_equal_output"] = len(set(outs.values())) == 1
    res["scaling_8_over_1"] = res["threads_8"]["blocks_per_s"] / res["threads_1"]["blocks_per_s"]
    return res


def encode_leg(args, plan, luma, chroma, world, dev):
    """the encoder over the frame stream -- dctq_encode_planes16
    (2-byte symbols, where the plan admits them; else dctq_encode_planes) (forward + zigzag run-length symbols of reference semantics, the symbol count
    fused into the forward launch) -- and at N>1 the all-gather of every rank's
    symbol stream (shard.gather_symbols), end to end, max over ranks.  Reports the
    stream size against the int16 coefficient planes (the bench's uniform input
    is the RLE worst case: most coefficients are nonzero)."""
    import ctypes as C
    from dct_amd import shard
    L = dct_amd.lib()
    pls = [luma, chroma]
    descs = (dct_amd._Plane * 2)(*[dct_amd.plane_desc(p) for p in pls])
    nbs = [p.shape[0] * (p.shape[1] // 8) * (p.shape[2] // 8) for p in pls]
    n = sum(nbs)
    # the planes' coefficients back to back in one allocation: the encoder writes each plane's
    # part, and the Huffman sizes of the whole step are then ONE launch over all n blocks
    coef_all = torch.empty((n, 64), dtype=torch.int16, device=dev)
    coefs = [coef_all[:nbs[0]], coef_all[nbs[0]:]]
    off = torch.empty(n + 1, dtype=torch.int32, device=dev)
    cap = 64 * n
    sb = plan.symbol_bytes  # 2 when the plan bounds every |quantized coefficient| by 511 (q <= 90)
    enc = L.dctq_encode_planes16 if sb == 2 else L.dctq_encode_planes  # the opt-in 2-byte format where admitted
    sym = torch.empty(cap, dtype=torch.int16 if sb == 2 else torch.int32, device=dev)
    ws = torch.empty(int(L.dctq_encode_workspace_bytes(n)) // 4 + 1, dtype=torch.int32, device=dev)
    cp = (C.c_void_p * 2)(*[c.data_ptr() for c in coefs])
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)

    def encode():
        rc = enc(plan._h, descs, 2, C.cast(cp, C.c_void_p), C.c_void_p(off.data_ptr()),
                 C.c_void_p(sym.data_ptr()), cap, C.c_void_p(ws.data_ptr()), stream)
        if rc:
            raise RuntimeError(f"dctq_encode_planes{'16' if sb == 2 else ''} rc={rc}")

    def timed(fn):
        return timed_steady(fn, args.encode_steps, dev)

    el = timed(encode)
    total = int(off[n].item()) & 0xFFFFFFFF
    out = {"op": "encode_planes (forward + zigzag/RLE, count fused) over all planes", "steps": args.encode_steps,
           "blocks_per_s": world * n * args.encode_steps / el, "ms_per_step": el / args.encode_steps * 1e3,
           "symbol_bytes": sb, "symbols_per_block": total / n, "stream_bytes_per_block": 4.0 + sb * total / n,
           "coefficient_bytes_per_block": 128}
    # the reference pipeline's per-block Huffman size (get_encoded_size after
    # build_huffman_codes, tests/test_entropy.c:329-341) of every block just encoded
    bits_all = torch.empty(n, dtype=torch.int32, device=dev)
    bits = [bits_all[:nbs[0]], bits_all[nbs[0]:]]

    def huffman():
        dct_amd.huffman_bits(coef_all, out=bits_all)  # one launch over both planes' blocks

    el_h = timed(huffman)
    mean_bits = float(sum(b.double().sum().item() for b in bits)) / n
    k = 240 * 135  # first chroma plane: checked against the oracle in the CPU leg (cpu_leg)
    huf_check = (coefs[1][:k].cpu().numpy(), bits[1][:k].cpu().numpy())
    out["huffman"] = {"op": "huffman_bits (per-block Huffman size, reference get_encoded_size) over all planes "
                            "(one launch over the step's coefficient stack)",
                      "blocks_per_s": world * n * args.encode_steps / el_h,
                      "ms_per_step": el_h / args.encode_steps * 1e3, "bits_per_block": mean_bits,
                      "compression_vs_u8": 512.0 / mean_bits, "_check": huf_check}
    # the same sizes straight from the pixels in one launch (coefficients on chip)
    fused_bits = torch.empty(n, dtype=torch.int32, device=dev)

    def huffman_from_pixels():
        rc = L.dctq_huffman_bits_planes(plan._h, descs, 2, C.c_void_p(fused_bits.data_ptr()), stream)
        if rc:
            raise RuntimeError(f"dctq_huffman_bits_planes rc={rc}")

    el_f = timed(huffman_from_pixels)
    out["huffman_from_pixels"] = {
        "op": "huffman_bits_planes (forward + quantization + per-block Huffman size in one launch) over all planes",
        "blocks_per_s": world * n * args.encode_steps / el_f, "ms_per_step": el_f / args.encode_steps * 1e3,
        "hbm_bytes_per_block": 68,
        "equals_forward_then_huffman_bits": bool(torch.equal(fused_bits, torch.cat(bits)))}
    def symbol_gather_leg():
        """N>1, run by main() among the all-gather legs: encode + the symbol streams all-gathered."""
        def encode_gather():
            encode()
            return shard.gather_symbols(off, sym)  # 4 B per block + sb B per symbol on the wire
        el2 = timed(encode_gather)
        return {"gather_op": "encode + symbol-stream all_gather ("
                             + ("RCCL" if dist.get_backend() == "nccl" else dist.get_backend()) + ")",
                "gather_blocks_per_s": world * n * args.encode_steps / el2,
                "gather_ms_per_step": el2 / args.encode_steps * 1e3}

    out["_symbol_gather_leg"] = symbol_gather_leg if dist.is_initialized() else None
    return out


LEG_PREWARM_MS = 30.0


def timed_steady(fn, steps, dev, prewarm_ms=LEG_PREWARM_MS):
    """Wall time of `steps` back-to-back calls of a secondary leg's step, measured
    the way the headline is (main()): the step first runs back to back, untimed,
    for about `prewarm_ms` -- between legs the GPU idles while the host works, and
    an idle MI355X drops its clocks within milliseconds (HISTORY.md 3.1b) -- then the
    timed steps are bracketed by a barrier and a synchronize on both sides; the
    max over ranks.  The pre-warm is a COUNT of calls that every rank agrees on
    (one timed call, the max over ranks of the count it suggests): a step may hold
    collectives (the symbol-stream gather), so every rank must call it equally often."""
    torch.cuda.synchronize()
    t = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    one = max(time.perf_counter() - t, 1e-6)
    n_pre = min(400, max(1, int(prewarm_ms * 1e-3 / one)))
    if dist.is_initialized():
        n = torch.tensor([n_pre], dtype=torch.int64, device=dev)
        dist.all_reduce(n, op=dist.ReduceOp.MAX)
        n_pre = int(n.item())
    for i in range(n_pre):
        fn()
        if i % 4 == 3:
            torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if dist.is_initialized():
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el


def round_trip_leg(args, plan, luma, chroma, world, rank, dev):
    """BASELINE configs[4]: forward DCT+quant then dequant+IDCT of every plane of
    the frame stream, FUSED (dctq_round_trip_planes: one launch, the quantized
    ints handed to the inverse through LDS, 448 B/block), end-to-end blocks/s
    (max over ranks) and PSNR of the first luma frame vs its input, with the
    reference's formula (recon clamped to [0,255], tests/test_entropy.c:376-393).
    The unfused pair (forward_quant_planes with var_num + dctq_inverse per plane,
    584 B/block) is timed alongside for comparison.  Non-adaptive plans reproduce
    the reference's 1/Q dequantization (src/quantization.c:139,144), hence their
    low PSNR."""
    import math
    pls = [luma, chroma]
    nbs = [px.shape[0] * (px.shape[1] // 8) * (px.shape[2] // 8) for px in pls]
    co = [torch.empty((n, 64), dtype=torch.int16, device=dev) for n in nbs]
    vn = [torch.empty(n, dtype=torch.int32, device=dev) for n in nbs]
    rec = [torch.empty((n, 64), dtype=torch.float32, device=dev) for n in nbs]

    def fused():
        plan.round_trip_planes(pls, outs=co, recons=rec)

    def unfused():
        plan.forward_quant_planes(pls, outs=co, var_nums=vn)
        for c, v, r in zip(co, vn, rec):
            plan.inverse(c, var_num=v, out=r)

    def timed(fn):
        return timed_steady(fn, args.round_trip_steps, dev)

    el_u = timed(unfused)
    el = timed(fused)  # rec / co hold the fused kernel's output from here on
    nblk = sum(nbs)
    # PSNR of luma frame 0 (block order is raster, so compare block by block)
    h, w = luma.shape[1], luma.shape[2]
    n0 = (h // 8) * (w // 8)
    orig = luma[0].reshape(h // 8, 8, w // 8, 8).permute(0, 2, 1, 3).reshape(n0, 64).double()

    def psnr_of(r):
        mse = float(((orig - r[:n0].double().clamp(0, 255)) ** 2).mean())
        return float("inf") if mse == 0 else 10.0 * math.log10(255.0 * 255.0 / mse)

    psnr = psnr_of(rec[0])
    # host copies for the CPU leg's oracle check (rank 0): chroma frame 0 -- its
    # pixels, the fused kernel's coefficients and recon -- and luma frame 0's PSNR
    nk = chroma.shape[1] // 8 * (chroma.shape[2] // 8)
    check = None
    if rank == 0:
        check = {"px": chroma[0].cpu().numpy(), "coef": co[1][:nk].cpu().numpy(), "recon": rec[1][:nk].cpu().numpy(),
                 "luma0": luma[0].cpu().numpy(), "psnr": psnr}
    movement = rt_ceiling_leg(args, plan, pls, co, rec, nblk, dev) if args.ceiling_rounds > 0 else None
    # the other dequantization semantics on the same frame: adaptive plans dequantize
    # with Q (src/quantization.c:137,144), non-adaptive ones with the reference's 1/Q
    other = dct_amd.Plan(args.quality, 0 if args.adaptive else 1)
    (_,), (r_other,) = other.round_trip_planes([luma[0]])
    psnr_other = psnr_of(r_other)
    bpb = 64 + 128 + 256
    inv_bound, inv_f32 = dct_amd.inverse_bound(args.quality, args.adaptive)
    return {"op": "round_trip_planes (fused forward+inverse, one launch per step; BASELINE configs[4])",
            "kernel": "roundtrip8<..., INV32=true> (paired-lane fp32 inverse)" if inv_f32 else "roundtrip8 (paired-lane fp64 inverse)",
            "inverse": {"arithmetic": "fp32" if inv_f32 else "fp64",
                        "error_bound": inv_bound if inv_f32 else None,
                        "rule": "fp32 when the rigorous bound of tools/inv_bound.py for this plan is <= 5e-5 "
                                "(non-adaptive plans; q <= 71 of the standard table), else the paired fp64 inverse"},
            "world_size": world, "scaling": "weak", "frames_per_gpu": luma.shape[0], "steps": args.round_trip_steps,
            "blocks_per_s": world * nblk * args.round_trip_steps / el,
            "ms_per_step": el / args.round_trip_steps * 1e3,
            "bytes_per_block": bpb, "achieved_GBs_per_gpu": nblk * bpb * args.round_trip_steps / el / 1e9,
            "frac_of_hbm_peak": nblk * bpb * args.round_trip_steps / el / 1e9 / HBM_PEAK_GBS,
            "movement_ceiling": movement,
            "unfused_blocks_per_s": world * nblk * args.round_trip_steps / el_u,
            "unfused_bytes_per_block": 64 + 128 + 4 + 128 + 4 + 256,
            "psnr_db_luma_frame0": psnr,
            f"psnr_db_luma_frame0_adaptive{0 if args.adaptive else 1}": psnr_other,
            "psnr_note": "adaptive=0 dequantizes with the reference's 1/Q (bug-compatible, src/quantization.c:139,144); "
                         "adaptive=1 with Q*(2-nv)", "_check": check}


def rt_ceiling_leg(args, plan, pls, co, rec, nblk, dev, b2b=3):
    """Memory ceilings of the fused round trip's traffic (64 B in, 128 + 256 B out
    per block) on THIS box, in interleaved steady-state rounds beside the fused
    launch itself (as ceilings_leg does for the forward):
      movement : dctq_diag_rt_movement_planes -- roundtrip8's exact grid, stage,
                 prefetch and stores, no arithmetic;
      flat_124 : dctq_diag_stream 5 -- the same byte counts as a flat persistent
                 stream (1 KiB loads, 24 x 1 KiB nt stores per 64 blocks) over the
                 workload's own pixel bytes (flat_124_const: over a constant buffer,
                 as rounds 3-5 measured it);
      flat_124_x32: dctq_diag_stream 16 -- the same bytes in the round trip's two output
                 arrays with its three drained store groups, on the round trip's grid
                 (32 x the resident workgroups): the faster flat stream on the boxes
                 measured (profiles/r06/rt_grid_ab); fused_over_flat_124 is taken against
                 the better of the two flat streams;
      plane_124: dctq_diag_stream 17 -- flat_124_x32 with the round trip's READ shape: each
                 lane loads its block's 8 rows (8 B each) from a 3840-px-wide plane, on the
                 same grid: the no-arithmetic ceiling of a block transform over image planes
                 (profiles/r06/INDEX.md, rt_read_shape_ab, rt_grid_ab).
    fused_over_own_movement is the kernel's time against its own data movement.
    Overwrites co/rec (run after the parity copies)."""
    import statistics
    D = dct_amd.diag()
    dplan = dct_amd.Plan(args.quality, args.adaptive, diagnostic=True)
    nflat = nblk // 64 * 64
    # the flat stream reads THE SAME PIXEL BYTES as the fused kernel (the luma and chroma stacks
    # back to back), as the forward's ceilings leg does: HBM moves constant data faster than
    # random data (up to 9 %, HISTORY.md 3.1b), and the stream's stores write what it read, so a
    # constant source inflates the ceiling.  Rounds 3-5 read a constant buffer here; that
    # variant is kept as flat_124_const (not a ceiling of this workload).
    src = torch.cat([p.reshape(-1) for p in pls])[:nflat * 64].contiguous()
    src7 = torch.full((nflat * 64,), 7, dtype=torch.uint8, device=dev)
    dst = torch.empty(nflat * 384, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream().cuda_stream

    def flat(buf, kind=5):
        rc = D.dctq_diag_stream(kind, buf.data_ptr(), dst.data_ptr(), nflat, stream)
        if rc:
            raise RuntimeError(f"dctq_diag_stream({kind}) rc={rc}")

    bpb = 64 + 128 + 256
    cases = {"fused": (lambda: plan.round_trip_planes(pls, outs=co, recons=rec), nblk * bpb),
             "movement": (lambda: dplan.diag_rt_movement_planes(pls, co, rec), nblk * bpb),
             "flat_124": (lambda: flat(src), nflat * bpb),
             "flat_124_const": (lambda: flat(src7), nflat * bpb),
             "flat_124_x32": (lambda: flat(src, 16), nflat * bpb),
             "plane_124": (lambda: flat(src, 17), nflat * bpb)}
    times = {k: [] for k in cases}
    for r in range(args.ceiling_rounds + 1):
        for k, (fn, _) in cases.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            fn()
            e0.record()
            for _ in range(b2b):
                fn()
            e1.record()
            torch.cuda.synchronize()
            if r:
                times[k].append(e0.elapsed_time(e1) * 1e-3 / b2b)
    med = {k: statistics.median(v) for k, v in times.items()}
    frac = {k: cases[k][1] / med[k] / 1e9 / HBM_PEAK_GBS for k in cases}
    del src, src7, dst
    best_flat = max(frac["flat_124"], frac["flat_124_x32"])
    return {"fused_frac": frac["fused"], "movement_frac": frac["movement"], "flat_124_frac": frac["flat_124"],
            "flat_124_x32_frac": frac["flat_124_x32"], "flat_124_const_frac": frac["flat_124_const"],
            "plane_124_frac": frac["plane_124"],
            "fused_over_plane_124": frac["fused"] / frac["plane_124"],
            "fused_over_own_movement": frac["fused"] / frac["movement"],
            "fused_over_flat_124": frac["fused"] / best_flat,
            "fused_over_flat_124_const": frac["fused"] / frac["flat_124_const"], "rounds": args.ceiling_rounds,
            "launches_per_sample": b2b, "median_us": {k: v * 1e6 for k, v in med.items()}}


def ceilings_leg(args, plan, luma, chroma, coef_y, coef_c, dev, rounds=10, b2b=3):
    """Memory ceilings of the forward kernel's traffic on THIS box, measured in
    rounds beside the forward launch itself, through the diagnostic library
    (libdct_amd_diag.so, csrc/dctq_diag.h):
      movement_v3 : dctq_diag_movement_planes -- the product kernel's (fdct8_quant_v3)
                    exact data movement (same grid, LDS footprint, prefetch, LDS
                    stage, 1 KiB stores), no math;
      movement_v3_x8 : the same pattern on the round-3 grid (8 x the resident workgroups,
                    dctq_diag_movement_grid_planes): without the arithmetic's latency slack the
                    16x grid's short-lived waves can move the same bytes slower on some boxes
                    (profiles/r04/movement_v3_grid_ab.log), so both grids are ceiling candidates;
      movement_v2 : dctq_diag_movement_v2_planes -- the same for fdct8_quant_v2 (the
                    tie-heavy plans' queue kernel), an extra named ceiling;
      flat_1to2_* : dctq_diag_stream 0/1/6/7 -- the same byte counts as a flat stream
                    (16 B per lane, 1 KiB per instruction), nt / default stores, on the
                    resident grid and on 16x / 32x grids (_x16, _x32: the grid the
                    forward runs, and twice it),
                    reading THE SAME PIXEL BYTES (the luma and chroma stacks back to
                    back): HBM moves constant data faster than random data (up to
                    9 %, HISTORY.md 3.1b), so a ceiling over a constant buffer is not a
                    ceiling of this workload -- flat_1to2_nt_nt_const shows that
                    effect and is not a candidate ceiling;
      plane_1to2_x32 : dctq_diag_stream 14 -- flat_1to2_nt_nt_x32's stores with the
                    forward's READ shape (each lane its block's 8 rows, 8 B each, from
                    a 3840-px-wide plane): the no-arithmetic ceiling of a block
                    transform over image planes, reported as forward_over_plane_1to2
                    (not a candidate for `pattern`: it is a model of the workload's
                    reads, profiles/r06/INDEX.md rt_read_shape_ab);
      read_only, write_only(_nt) : dctq_diag_stream 2/3/4 over the same byte counts;
      phased_*    : a read-only launch then a write-only launch, timed as a pair,
                    i.e. the 1:2 traffic with no mix (not reachable by one launch
                    that transforms the data: profiles/r02/hbm_ceilings.md).
    Steady state: every sample is `b2b` launches of one case back to back after
    one untimed launch of the same case.  Default-policy stores leave dirty lines
    in the caches that are written back during the NEXT launch, so timing single
    launches in rotation charges one case's write-back to another (round 2:
    plain stores looked 2-25 % faster than nt that way and were 4-15 % slower
    in steady state, profiles/r02/policy_b2b.md).
    movement_ceiling = the best 1:2 pattern; the forward kernel's time against
    it is forward_over_ceiling.  Overwrites coef_y/coef_c (run after the parity
    check)."""
    import statistics
    D = dct_amd.diag()
    dplan = dct_amd.Plan(args.quality, args.adaptive, diagnostic=True)
    pls, outs = [luma, chroma], [coef_y, coef_c]
    nblk = coef_y.shape[0] + coef_c.shape[0]
    nflat = nblk // 64 * 64
    src = torch.cat([luma.reshape(-1), chroma.reshape(-1)])[:nflat * 64].contiguous()  # the workload's pixels
    src7 = torch.full((nflat * 64,), 7, dtype=torch.uint8, device=dev)  # constant data (rounds 1-3's flat input)
    dst = torch.empty(nflat * 128, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream().cuda_stream

    def diag_stream(*kinds, buf=src):
        for kind in kinds:
            rc = D.dctq_diag_stream(kind, buf.data_ptr(), dst.data_ptr(), nflat, stream)
            if rc:
                raise RuntimeError(f"dctq_diag_stream({kind}) rc={rc}")

    cases = {
        "forward": (lambda: plan.forward_quant_planes(pls, outs=outs), nblk * BYTES_PER_BLOCK),
        "movement_v3": (lambda: dplan.diag_movement_planes(pls, outs), nblk * BYTES_PER_BLOCK),
        "movement_v3_x8": (lambda: dplan.diag_movement_planes(pls, outs, grid_mult=8), nblk * BYTES_PER_BLOCK),
        "movement_v2": (lambda: dplan.diag_movement_planes(pls, outs, shape=2), nblk * BYTES_PER_BLOCK),
        "flat_1to2_nt_nt": (lambda: diag_stream(0), nflat * BYTES_PER_BLOCK),
        "flat_1to2_nt_nt_x16": (lambda: diag_stream(6), nflat * BYTES_PER_BLOCK),
        "flat_1to2_nt_nt_x32": (lambda: diag_stream(7), nflat * BYTES_PER_BLOCK),
        "flat_1to2_nt_nt_const": (lambda: diag_stream(0, buf=src7), nflat * BYTES_PER_BLOCK),
        "plane_1to2_x32": (lambda: diag_stream(14), nflat * BYTES_PER_BLOCK),
        "flat_1to2_nt_plain": (lambda: diag_stream(1), nflat * BYTES_PER_BLOCK),
        "read_only": (lambda: diag_stream(2), nflat * 64),
        "write_only": (lambda: diag_stream(3), nflat * 128),
        "write_only_nt": (lambda: diag_stream(4), nflat * 128),
        "phased_read_then_write": (lambda: diag_stream(2, 3), nflat * BYTES_PER_BLOCK),
        "phased_read_then_write_nt": (lambda: diag_stream(2, 4), nflat * BYTES_PER_BLOCK),
    }
    times = {k: [] for k in cases}
    for r in range(rounds + 1):
        for k, (fn, _) in cases.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            fn()  # the sample's predecessor is the same case
            e0.record()
            for _ in range(b2b):
                fn()
            e1.record()
            torch.cuda.synchronize()
            if r:
                times[k].append(e0.elapsed_time(e1) * 1e-3 / b2b)
    med = {k: statistics.median(v) for k, v in times.items()}
    frac = {k: cases[k][1] / med[k] / 1e9 / HBM_PEAK_GBS for k in cases}
    best = max(("movement_v3", "movement_v3_x8", "flat_1to2_nt_nt", "flat_1to2_nt_nt_x16", "flat_1to2_nt_nt_x32", "flat_1to2_nt_plain"),
               key=lambda k: frac[k])
    del src, src7, dst
    return {"pattern": best, "achieved": frac[best] * HBM_PEAK_GBS, "frac": frac[best],
            "forward_frac": frac["forward"], "forward_over_ceiling": frac["forward"] / frac[best],
            "forward_over_own_movement": frac["forward"] / frac["movement_v3"],
            "forward_over_plane_1to2": frac["forward"] / frac["plane_1to2_x32"], "rounds": rounds,
            "launches_per_sample": b2b,
            "hw_ceilings": {k: {"median_us": med[k] * 1e6, "frac": frac[k],
                                **({"note": "two kernels: an upper bound no single launch that transforms the "
                                            "data reaches"} if k.startswith("phased") else {})}
                            for k in cases}}


def build_record():
    """Which library this line measured: the sha256 of the loaded libdct_amd.so
    and whether it is the one dct_amd/build.py's manifest (build_info.json:
    sha256 of every source it was built from) says it built."""
    import hashlib
    from dct_amd import build as B
    sha = hashlib.sha256(open(dct_amd.LIB_PATH, "rb").read()).hexdigest()
    info = B.build_info()
    return {"lib_sha256": sha, "manifest_lib_sha256_matches": info.get("lib_sha256") == sha,
            "built_utc": info.get("built_utc"), "hipcc": info.get("hipcc")}


def traffic_for(args, launches):
    """PMC HBM traffic of this exact configuration, or None with the reason: the
    stored measurement (tools/pmc_traffic.py) must match frames, kind, quality,
    adaptive mode, launches per step and the sha256 of the libdct_amd.so that
    is loaded now."""
    import hashlib
    if not os.path.exists(args.traffic):
        return None, "no profiles/traffic.json"
    try:
        tj = json.load(open(args.traffic))
    except (OSError, ValueError) as e:
        return None, f"unreadable traffic file: {e}"
    lib_sha = hashlib.sha256(open(dct_amd.LIB_PATH, "rb").read()).hexdigest()
    want = {"frames": args.frames, "kind": args.kind, "quality": args.quality, "adaptive": args.adaptive,
            "launches_per_step": launches, "lib_sha256": lib_sha}
    bad = [k for k, v in want.items() if tj.get(k) != v]
    if bad:
        return None, "stored PMC traffic does not match this run (" + ", ".join(bad) + ")"
    return tj.get("bytes_per_launch"), "PMC FETCH_SIZE x 2 + WRITE_SIZE (tools/pmc_traffic.py)"


def main():
    args = parse()
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))  # one child process per GPU; this process stays off the GPU
    if int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={os.environ.get('WORLD_SIZE')} "
                 "ranks")
    if args.launch_check:
        return launch_check(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # --dist-legs at one process: a one-rank process group over the chosen backend,
    # so the N>1 legs (RCCL all-gathers of coefficients and symbol streams, the band
    # split) run end to end on a single GPU (tests/test_gpu_parity.py)
    dist_on = world > 1 or args.dist_legs
    if dist_on and world == 1:
        import socket
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(sk.getsockname()[1]))
        sk.close()
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if dist_on:
        import datetime
        # a collective still waiting on a peer after --dist-timeout raises in the CALLER (the
        # optional legs catch it, class Legs): for RCCL that is TORCH_NCCL_BLOCKING_WAIT=1 -- the
        # waiting call blocks the host until the work completes or the timeout passes, then
        # throws, and torch creates no watchdog thread that would tear the process down instead
        # (DESIGN 7); gloo raises at the timeout by itself
        if args.backend == "nccl":
            os.environ.setdefault("TORCH_NCCL_BLOCKING_WAIT", "1")
        local = local % max(1, torch.cuda.device_count())  # rehearsal: several ranks may share a GPU
        torch.cuda.set_device(local)
        timeout = datetime.timedelta(seconds=args.dist_timeout)
        with _StdoutToStderr():
            if args.backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=timeout)
            else:
                dist.init_process_group(args.backend, timeout=timeout)
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)
    if dist_on:
        world = dist.get_world_size()  # echo the process group's size, not only the launcher's env
    F = args.frames
    seed = args.seed + 100000 * rank

    # ---- inputs resident in HBM (synthesised on the device)
    luma = dct_amd.synth(seed, args.kind, Y_W, Y_H, F, device=dev)
    chroma = dct_amd.synth(seed + 50000, args.kind, C_W, C_H, 2 * F, device=dev)
    nblk_y = F * (Y_W // 8) * (Y_H // 8)
    nblk_c = 2 * F * (C_W // 8) * (C_H // 8)
    coef_y = torch.empty((nblk_y, 64), dtype=torch.int16, device=dev)
    coef_c = torch.empty((nblk_c, 64), dtype=torch.int16, device=dev)
    plan = dct_amd.Plan(args.quality, args.adaptive)
    torch.cuda.synchronize()

    launches = 2 if args.per_plane else 1

    def step():
        if args.per_plane:
            plan.forward_quant(luma, out=coef_y)
            plan.forward_quant(chroma, out=coef_c)
        else:
            plan.forward_quant_planes([luma, chroma], outs=[coef_y, coef_c])

    # Clock ramp: from idle, the first ~50 launches (~25 ms) run up to 20 % slower
    # than the steady state (tools/ramp.py).  A serving GPU is not idle, so the
    # step runs back to back untimed until `prewarm_ms` of it has executed, then
    # the W warmup steps, then the K timed steps.
    prewarm_steps, t_pre = 0, time.perf_counter()
    while args.prewarm_ms > 0 and (time.perf_counter() - t_pre) * 1e3 < args.prewarm_ms:
        for _ in range(8):
            step()
        prewarm_steps += 8
        torch.cuda.synchronize()  # the time bound counts executed work, not queued launches
    prewarm = {"steps": prewarm_steps, "ms": (time.perf_counter() - t_pre) * 1e3}
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # HIP events on the launch stream bracket the K launches as a whole: an event
    # record between launches costs ~2-3 us of GPU time each (tools/event_overhead.py:
    # two per step took 1.6 % off the step rate), so none sits inside the region.
    # The average launch duration below therefore includes the K-1 launch gaps
    # (~2 us each), i.e. it is slightly conservative against rocprofv3's.
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    for k in range(args.steps):
        step()
    ev1.record()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if dist_on:
        dist.barrier()
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    # mean launch duration over the timed region (HIP events on the launch stream)
    avg_launch_s = ev0.elapsed_time(ev1) * 1e-3 / (launches * args.steps)
    avg_launch_bytes = BYTES_PER_BLOCK * (nblk_y + nblk_c) / launches
    achieved = avg_launch_bytes / avg_launch_s / 1e9

    # host copies of one chroma plane and its coefficients: the CPU leg (rank 0)
    # checks them against the oracle
    fwd_check = None
    if rank == 0:
        nk = (C_W // 8) * (C_H // 8)
        fwd_check = (chroma[0].cpu().numpy(), coef_c[:nk].cpu().numpy())
    trace("headline done")

    # ---- the line, headline first: every optional leg below only adds to it
    total_blocks = world * (nblk_y + nblk_c) * args.steps
    traffic, traffic_note = traffic_for(args, launches)
    report = Report(rank)
    out = {
        "metric": "8x8 macroblocks/sec (DCT+quant); % HBM roofline",
        "value": total_blocks / el,
        "unit": "macroblocks/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "prewarm": prewarm,
        "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (device splitmix64 frames, kind=%s)" % args.kind,
        "config": {"workload": f"4K 4:2:0 frame stream (BASELINE configs[2] planes), {F} frames/GPU/step, "
                               f"forward DCT+quant q{args.quality} adaptive={args.adaptive}, int16 out",
                   "frames_per_gpu": F, "blocks_per_gpu_step": nblk_y + nblk_c, "quality": args.quality,
                   "adaptive": args.adaptive, "parallelism": f"frames sharded over {world} GPU(s)",
                   "world_size": world, "backend": dist.get_backend() if dist_on else None},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_note,
                     "kernel": dct_amd.forward_kernel(args.quality, args.adaptive,
                                                      -(-nblk_y // 64) + -(-nblk_c // 64),
                                                      torch.cuda.get_device_properties(dev).multi_processor_count),
                     "avg_launch_us": avg_launch_s * 1e6, "launches_per_step": launches,
                     "bytes_per_launch": avg_launch_bytes, "movement_ceiling": None},
        "cpu_baseline": None, "parity_check": None, "parity_error": None,
        "gather": None, "band": None, "round_trip": None, "encode": None, "small_frame": None,
        "legacy_per_block": None,
        "gpu": None, "build": build_record(),
        "note": "u8 pixels in, int16 coefficients out; fp32 AAN butterfly with the exact fp64 "
                "reference-order recomputation for guard-band (tie) coefficients",
    }
    report.out = out
    legs = Legs(report, dist_on, args.leg_deadline or 2 * args.dist_timeout + 60.0)
    out["legs"] = legs.status

    # ---- optional legs, fail-soft (class Legs): this rank's own work first, then the
    # legs whose steps hold all-gathers, then the direct-push (p2p) legs last
    if args.ceiling_rounds > 0 and not args.per_plane:
        out["roofline"]["movement_ceiling"] = legs.run(
            "ceilings", lambda: ceilings_leg(args, plan, luma, chroma, coef_y, coef_c, dev, args.ceiling_rounds),
            collective=False)
    if world == 1 and not args.no_cpu:  # single-GPU config
        out["small_frame"] = legs.run("small_frame", lambda: small_frame_leg(args, plan, dev), collective=False)
        out["legacy_per_block"] = legs.run("legacy_per_block", lambda: legacy_leg(args, dev), collective=False)
    encode = None
    if args.encode_steps > 0:  # its timing takes the max over ranks: collective at N>1
        encode = legs.run("encode", lambda: encode_leg(args, plan, luma, chroma, world, dev))
    round_trip = None
    if args.round_trip_steps > 0:
        round_trip = legs.run("round_trip", lambda: round_trip_leg(args, plan, luma, chroma, world, rank, dev))
    # host copies for the CPU leg's oracle checks come off the leg results at once: the
    # line may be printed (watchdog) at any point from here on
    huf_check = encode["huffman"].pop("_check", None) if encode else None
    rt_check = round_trip.pop("_check", None) if round_trip else None
    symbol_gather = encode.pop("_symbol_gather_leg", None) if encode else None
    out["encode"], out["round_trip"] = encode, round_trip
    gather_parts, band_parts = {}, {}
    if dist_on and args.gather_steps > 0:
        gather_parts["all_gather"] = legs.run(
            "gather.all_gather", lambda: gather_leg(args, plan, world, rank, dev, ("all_gather",)))
        band_parts["all_gather"] = legs.run(
            "band.all_gather", lambda: band_leg(args, plan, luma, chroma, world, dev, ("all_gather",)))
    if symbol_gather is not None:
        sg = legs.run("encode.symbol_gather", symbol_gather)
        encode.update(sg or {"gather_error": legs.status["encode.symbol_gather"]})
    if dist_on and args.gather_steps > 0:
        gather_parts["p2p"] = legs.run("gather.p2p", lambda: gather_leg(args, plan, world, rank, dev, ("p2p",)))
        band_parts["p2p"] = legs.run("band.p2p", lambda: band_leg(args, plan, luma, chroma, world, dev, ("p2p",)))
        out["gather"] = merge_methods(gather_parts["all_gather"], gather_parts["p2p"], "p2p",
                                      legs.status.get("gather.p2p"))
        out["band"] = merge_methods(band_parts["all_gather"], band_parts["p2p"], "p2p",
                                    legs.status.get("band.p2p"))
        if out["gather"] is not None:
            out["gather"].setdefault("fault_injected", args.gather_fault)
    trace("legs done")

    if rank == 0:
        if not args.no_cpu:
            res = legs.run("cpu", lambda: cpu_leg(args, world, fwd_check, huf_check, rt_check), collective=False)
            cpu, parity = res if res is not None else (None, None)
            out["cpu_baseline"] = cpu
            lp = out.get("legacy_per_block")
            if cpu and lp:  # the stated baseline beside it: the reference's own loop on one CPU thread
                lp["reference_cpu_one_thread_blocks_per_s"] = cpu["builds"]["O2_one_thread"]["blocks_per_s"]
            if parity is not None:
                out["parity_check"], out["parity_error"] = parity.get("forward"), parity.get("error")
                if encode:
                    encode["huffman"]["parity_check_chroma0"] = parity.get("huffman")
                if round_trip and "round_trip" in parity:
                    rp = parity["round_trip"]
                    round_trip["parity"] = rp
                    round_trip["parity_check"] = bool(rp["coef_bit_exact"] and rp["recon_within_1e-4"]
                                                      and rp["psnr_abs_diff"] <= 1e-3)
        out["gpu"] = gpu_identity()
    report.emit()
    if dist_on:
        if legs.poisoned:
            # a collective this rank gave up on may still be queued on its stream: leave
            # without tearing the group down (destroy would wait on it)
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(0)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
