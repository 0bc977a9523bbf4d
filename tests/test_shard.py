"""CPU, world_size 2 and 3 over gloo: the multi-GPU partitioning (dct_amd/shard.py).

Each rank transforms only its shard -- here with the oracle standing in for
the device kernel, since this container has no GPU (the -m gpu tests prove the
kernel equals the oracle) -- then the coefficient shards are all-gathered and
every rank checks the result equals the unsharded plane's coefficients in the
reference's raster block order."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dct_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import oracle as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # (1) frame shards of a ragged batch: 5 frames of 48x40
        frames = torch.from_numpy(np.stack([O.synth_plane(7 + f, O.KINDS["uniform"], 48, 40) for f in range(5)]))
        mine, (lo, hi) = shard.frame_shard(frames, world, rank)
        local = torch.from_numpy(np.concatenate([O.forward_plane(f.numpy(), 50, 0) for f in mine])
                                 if hi > lo else np.zeros((0, 64), np.int16))
        per = (48 // 8) * (40 // 8)
        counts = [(shard.split(5, world, r)[1] - shard.split(5, world, r)[0]) * per for r in range(world)]
        want = np.concatenate([O.forward_plane(f.numpy(), 50, 0) for f in frames])
        for method in shard.GATHER_METHODS:  # the all-gather collective and the direct peer pushes
            full = shard.gather_coefficients(local, counts, method=method)
            assert np.array_equal(full.numpy(), want), f"frame-sharded gather differs ({method})"

        # (2) block-row bands of one plane: 7 block rows, adaptive, q90
        plane = torch.from_numpy(O.synth_plane(99, O.KINDS["smooth"], 64, 56))
        band, (row0, rows) = shard.band_shard(plane, world, rank)
        local = torch.from_numpy(O.forward_plane(np.ascontiguousarray(band.numpy()), 90, 1)
                                 if rows else np.zeros((0, 64), np.int16))
        counts = [shard.split(7, world, r)[1] * 8 - shard.split(7, world, r)[0] * 8 for r in range(world)]
        for method in shard.GATHER_METHODS:
            full = shard.gather_coefficients(local, counts, method=method)
            assert np.array_equal(full.numpy(), O.forward_plane(plane.numpy(), 90, 1)), f"band gather differs ({method})"

        # (2b) a frame's three planes in block-row bands, gathered in ONE collective (bench's band leg)
        planes = [O.synth_plane(500 + k, O.KINDS[kind], w, h)
                  for k, (kind, w, h) in enumerate([("uniform", 64, 56), ("smooth", 32, 24), ("extreme", 32, 24)])]
        locs, cnts = [], []
        for pl in planes:
            band, (row0, rows) = shard.band_shard(torch.from_numpy(pl), world, rank)
            locs.append(torch.from_numpy(O.forward_plane(np.ascontiguousarray(band.numpy()), 50, 0)
                                         if rows else np.zeros((0, 64), np.int16)))
            bh = pl.shape[0] // 8
            cnts.append([(b - a) * (pl.shape[1] // 8) for a, b in (shard.split(bh, world, r) for r in range(world))])
        for method in shard.GATHER_METHODS:
            fulls = shard.gather_planes(locs, cnts, method=method)
            for pl, f in zip(planes, fulls):
                assert np.array_equal(f.numpy(), O.forward_plane(pl, 50, 0)), f"multi-plane band gather differs ({method})"

        # (2c) direct pushes with EMPTY shards on some ranks (a 1-block-row plane: only rank 0 holds rows)
        tiny = O.synth_plane(901, O.KINDS["uniform"], 40, 8)
        band, (row0, rows) = shard.band_shard(torch.from_numpy(tiny), world, rank)
        local = torch.from_numpy(O.forward_plane(np.ascontiguousarray(band.numpy()), 50, 0)
                                 if rows else np.zeros((0, 64), np.int16))
        counts = [(b - a) * 5 for a, b in (shard.split(1, world, r) for r in range(world))]
        full = shard.gather_coefficients(local, counts, method="p2p")
        assert np.array_equal(full.numpy(), O.forward_plane(tiny, 50, 0)), "p2p gather with empty shards differs"
        with pytest.raises(ValueError):
            shard.gather_coefficients(local, counts, method="ring")

        # (2d) both shapes inside a SUBGROUP that excludes global rank 0: its ranks are not the
        # global ones, so the direct pushes must address peers by group rank
        sub_ranks = list(range(1, world)) if world > 2 else [0, 1]
        sub = dist.new_group(sub_ranks)  # collective over the world: every rank calls it
        if rank in sub_ranks:
            sw, sr = len(sub_ranks), sub_ranks.index(rank)
            mine, (lo, hi) = shard.frame_shard(frames, sw, sr)
            local = torch.from_numpy(np.concatenate([O.forward_plane(f.numpy(), 50, 0) for f in mine])
                                     if hi > lo else np.zeros((0, 64), np.int16))
            counts = [(shard.split(5, sw, r)[1] - shard.split(5, sw, r)[0]) * 30 for r in range(sw)]
            for method in shard.GATHER_METHODS:
                full = shard.gather_coefficients(local, counts, group=sub, method=method)
                assert np.array_equal(full.numpy(), want), f"subgroup gather differs ({method})"
        dist.barrier()

        # (3) run-length streams of the frame shards (what dctq_encode_planes makes on each GPU)
        mine, (lo, hi) = shard.frame_shard(frames, world, rank)
        local = (np.concatenate([O.forward_plane(f.numpy(), 50, 0) for f in mine])
                 if hi > lo else np.zeros((0, 64), np.int16))
        loff, lsym = O.rle_encode_plane(local)
        off, sym = shard.gather_symbols(torch.from_numpy(loff.view(np.int32)), torch.from_numpy(lsym.view(np.int32)))
        woff, wsym = O.rle_encode_plane(np.concatenate([O.forward_plane(f.numpy(), 50, 0) for f in frames]))
        assert np.array_equal(off.numpy().view(np.uint32), woff), "gathered offsets differ"
        assert np.array_equal(sym.numpy().view(np.uint32), wsym), "gathered symbols differ"
        # the 2-byte format (plans whose |q| <= 511, dctq_plan_symbol_bytes): same offsets, half the bytes
        off16, sym16 = shard.gather_symbols(torch.from_numpy(loff.view(np.int32)),
                                            torch.from_numpy(O.pack16(lsym).view(np.int16).copy()))
        assert sym16.dtype == torch.int16
        assert np.array_equal(off16.numpy().view(np.uint32), woff), "gathered offsets differ (2-byte)"
        assert np.array_equal(sym16.numpy().view(np.uint16), O.pack16(wsym)), "gathered 2-byte symbols differ"

        # (4) bench.py's N>1 gather leg (BASELINE configs[3], strong scaling) end to end:
        # shard.strong_gather_leg over a ragged frame split, the oracle standing in for the kernel
        total = 7
        lo, hi = shard.split(total, world, rank)
        stack = torch.from_numpy(np.stack([O.synth_plane(300 + f, O.KINDS["uniform"], 32, 24)
                                           for f in range(total)]))
        per = (32 // 8) * (24 // 8)
        counts = [(b - a) * per for a, b in (shard.split(total, world, r) for r in range(world))]

        def forward(fr):
            return torch.from_numpy(np.concatenate([O.forward_plane(f.numpy(), 75, 0) for f in fr])
                                    if fr.shape[0] else np.zeros((0, 64), np.int16))

        def unsharded():  # the whole stack's forward, recomputed here, in two pieces
            w = np.concatenate([O.forward_plane(f.numpy(), 75, 0) for f in stack])
            return [(0, torch.from_numpy(w[:5])), (5, torch.from_numpy(w[5:]))]

        r = shard.strong_gather_leg(forward, stack[lo:hi], counts, 2, torch.device("cpu"), unsharded=unsharded)
        for m, rm in r["by_method"].items():
            assert rm["gathered_equals_unsharded"] is True, m
        # a wrong shard offset shared by both gather shapes (every rank transforms the frames
        # one past its own slice): both shapes still agree with each other, the unsharded
        # check catches it on every rank
        shifted = stack[[(f + 1) % total for f in range(lo, hi)]]
        bad = shard.strong_gather_leg(forward, shifted, counts, 1, torch.device("cpu"), unsharded=unsharded)
        assert torch.equal(bad["by_method"]["p2p"]["full"], bad["by_method"]["all_gather"]["full"])
        assert not any(v["gathered_equals_unsharded"] for v in bad["by_method"].values()), rank
        assert not shard.equals_unsharded(torch.zeros(4, 64, dtype=torch.int16),
                                          [(0, torch.zeros(2, 64, dtype=torch.int16))])  # short cover
        assert r["blocks_per_step"] == total * per and r["steps"] == 2
        assert r["kernel_s"] > 0 and r["end_to_end_s"] > 0 and r["gather_s"] > 0
        assert set(r["by_method"]) == set(shard.GATHER_METHODS)
        for m, rm in r["by_method"].items():  # both shapes timed, both gather the same coefficients
            assert rm["end_to_end_s"] > 0 and rm["gather_s"] > 0
            assert torch.equal(rm["full"], r["full"]), m
        x = shard.xgmi_report((total * per - counts[rank]) * 128, r["gather_s"] / r["steps"], world)
        assert x["bytes_received_per_rank"] == (total * per - counts[rank]) * 128
        assert x["direct_estimate_GBs"] == (world - 1) * shard.XGMI_LINK_GBS
        assert abs(x["frac_of_direct_estimate"] * x["direct_estimate_GBs"] - x["achieved_GBs_per_rank"]) < 1e-9
        want = np.concatenate([O.forward_plane(f.numpy(), 75, 0) for f in stack])
        assert np.array_equal(r["full"].numpy(), want), "strong-scaling gather differs"
        assert np.array_equal(r["local"].numpy(), want[sum(counts[:rank]):sum(counts[:rank + 1])])
        q.put((rank, "ok"))
    except BaseException as e:  # noqa: BLE001 -- report to the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_gather_matches_unsharded(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {r: "ok" for r in range(world)}, res


def test_split_covers_exactly():
    for n in [0, 1, 7, 64, 270, 1000]:
        for world in [1, 2, 3, 8]:
            parts = [shard.split(n, world, r) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
            sizes = [hi - lo for lo, hi in parts]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard.split(4, 2, 2)
