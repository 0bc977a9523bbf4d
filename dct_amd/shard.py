"""Multi-GPU sharding of the DCT+quant path.

Blocks are independent (quantize reads only the plan and its own block,
src/quantization.c:113-131), so the path partitions with no data exchange:

* a batch of frames splits into contiguous frame ranges, one per rank;
* a single large plane splits into contiguous bands of block rows -- a band is
  itself a plane (pixel pointer advanced by 8*row0*stride, height 8*rows), and
  its coefficients are a contiguous slice of the raster-order output.

The only collectives are OPTIONAL gathers: of the int16 coefficient planes
(BASELINE configs[3]: "RCCL allgather of quantized coefficient planes over
xGMI"; several planes of a frame in one message with gather_planes), or of the
run-length symbol streams the encoder makes of them (shrink the
bytes before the exchange).  The ordering of the gathered result equals the
unsharded raster order, so rank r's slice lands at blocks_before(r).

The coefficient gathers come in SURVEY 8(e)'s two shapes (`method`):
  "all_gather" -- one all_gather_into_tensor per call over the whole shard,
                  padded to the largest shard so ragged splits work (RCCL picks
                  its algorithm: a ring takes in one xGMI link per step);
  "p2p"        -- direct pushes: every rank sends its shard to each of the
                  N - 1 peers and receives each peer's shard straight into its
                  slot of the output, all 2 (N - 1) transfers in ONE group
                  (dist.batch_isend_irecv = ncclGroupStart / ncclSend x (N-1) /
                  ncclRecv x (N-1) / ncclGroupEnd), so all 7 links of an MI355X
                  node carry data at once; no padding and no compaction copy.
The gathered tensors are identical either way (tests/test_shard.py).
"""
from __future__ import annotations


def split(n: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [lo, hi) share of n units for `rank`; the first n % world ranks get one more."""
    if world < 1 or not 0 <= rank < world or n < 0:
        raise ValueError("bad split arguments")
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def frame_shard(px, world: int, rank: int):
    """Frames [lo, hi) of a [F, H, W] stack owned by `rank` (a view, no copy)."""
    lo, hi = split(px.shape[0], world, rank)
    return px[lo:hi], (lo, hi)


def band_shard(px, world: int, rank: int):
    """Block-row band of one [H, W] plane owned by `rank` (a view, no copy).
    Returns (band, (row0, rows)) in block rows; the band's coefficients are
    coef[row0 * W/8 : (row0 + rows) * W/8] of the whole plane."""
    if px.shape[-2] % 8 or px.shape[-1] % 8:
        raise ValueError("plane dimensions must be multiples of 8")
    lo, hi = split(px.shape[-2] // 8, world, rank)
    return px[..., 8 * lo:8 * hi, :], (lo, hi - lo)


GATHER_METHODS = ("all_gather", "p2p")


def _check_method(method):
    if method not in GATHER_METHODS:
        raise ValueError(f"gather method must be one of {GATHER_METHODS}")


def _wire(t):
    """The bytes of a contiguous tensor as uint8 (RCCL has no int16; gloo moves raw bytes)."""
    import torch
    return t.reshape(-1).view(torch.uint8)


def gather_p2p(locals_, counts, group=None):
    """Direct-push gather of several planes' shards (SURVEY 8(e) "grouped
    ncclSend/ncclRecv"): locals_[p] is this rank's [counts[p][rank], ...] shard
    of plane p.  Every rank pushes each of its shards to every peer and receives
    every peer's shard directly into its row range of the per-plane output
    ([sum(counts[p]), ...], rank order), all transfers in one
    dist.batch_isend_irecv group -- N - 1 concurrent peer links, no padding,
    no staging buffer, no compaction.  Empty shards send nothing (both ends
    skip them).  The own shard is a device copy."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if len(locals_) != len(counts) or not locals_:
        raise ValueError("one counts list per plane")
    # gloo's send/recv move host memory only: device shards travel through host copies there
    # (the rehearsal of the N>1 legs on one GPU); RCCL moves them device to device over xGMI
    host = dist.get_backend(group) != "nccl" and locals_[0].device.type != "cpu"
    fulls, ops = [], []
    for loc, c in zip(locals_, counts):
        if len(c) != world or loc.shape[0] != c[rank]:
            raise ValueError("counts must list every rank's shard size of every plane")
        offs = [0]
        for n in c:
            offs.append(offs[-1] + n)
        dev = torch.device("cpu") if host else loc.device
        full = torch.empty((offs[-1],) + tuple(loc.shape[1:]), dtype=loc.dtype, device=dev)
        src = loc.to(dev).contiguous()
        full[offs[rank]:offs[rank + 1]].copy_(src)
        for d in range(1, world):  # peers in ring order from this rank: every link busy at once
            to, frm = (rank + d) % world, (rank - d) % world
            # group_peer: ranks within `group` (a subgroup's rank r is not global rank r)
            if c[rank]:
                ops.append(dist.P2POp(dist.isend, _wire(src), group=group, group_peer=to))
            if c[frm]:
                ops.append(dist.P2POp(dist.irecv, _wire(full[offs[frm]:offs[frm + 1]]), group=group, group_peer=frm))
        fulls.append(full)
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    if host:
        fulls = [f.to(loc.device) for f, loc in zip(fulls, locals_)]
    return fulls


def gather_coefficients(local, counts, group=None, method="all_gather"):
    """All-gather int16 coefficient shards [n_r, 64] (n_r = counts[r]) into the
    full [sum(counts), 64] tensor on every rank, in rank order.

    method "all_gather": one collective over the whole shard (bigger messages,
    fewer calls), ragged shards padded to max(counts) and compacted after the
    exchange.  method "p2p": gather_p2p's direct pushes."""
    import torch
    import torch.distributed as dist
    _check_method(method)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if len(counts) != world or local.shape[0] != counts[rank]:
        raise ValueError("counts must list every rank's shard size")
    if method == "p2p":
        return gather_p2p([local], [counts], group)[0]
    m = max(counts)
    if local.shape[0] < m:
        pad = torch.zeros((m - local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        send = torch.cat([local, pad])
    else:
        send = local.contiguous()
    if dist.get_backend(group) == "nccl":
        out = torch.empty((world * m,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        # RCCL has no int16 type: the same bytes as int32 (64 coefficients = 32 words a block)
        dist.all_gather_into_tensor(out.view(torch.int32), send.view(torch.int32), group=group)
        if all(c == m for c in counts):
            return out
        parts = list(out.split(m))
    else:  # gloo (CPU tests): no int16 reductions there, so move the raw bytes
        raw = send.view(torch.uint8)
        parts = [torch.empty_like(raw) for _ in range(world)]
        dist.all_gather(parts, raw, group=group)
        parts = [p.view(local.dtype) for p in parts]
    if all(c == m for c in counts):
        return torch.cat(parts)
    return torch.cat([p[:c] for p, c in zip(parts, counts)])


def gather_planes(locals_, counts, group=None, method="all_gather"):
    """All-gather the coefficient shards of SEVERAL planes (e.g. a frame's Y, Cb
    and Cr bands: locals_[p] is [counts[p][rank], 64]) in ONE collective: every
    plane's shard padded to its largest rank, concatenated, exchanged, and split
    back into per-plane [sum(counts[p]), 64] tensors in rank order.  One message
    instead of one per plane: each collective pays the RCCL launch and ring
    latency, and a 4K frame's band is only ~2-4 MB per rank at N = 8.
    method "p2p": every plane's shard pushed to every peer in one group
    (gather_p2p), received in place."""
    import torch
    import torch.distributed as dist
    _check_method(method)
    if method == "p2p":
        return gather_p2p(locals_, counts, group)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if len(locals_) != len(counts) or not locals_:
        raise ValueError("one counts list per plane")
    for loc, c in zip(locals_, counts):
        if len(c) != world or loc.shape[0] != c[rank]:
            raise ValueError("counts must list every rank's shard size of every plane")
    ms = [max(c) for c in counts]
    ref = locals_[0]
    pieces = []
    for loc, m in zip(locals_, ms):
        pieces.append(loc.contiguous())
        if loc.shape[0] < m:
            pieces.append(torch.zeros((m - loc.shape[0],) + tuple(ref.shape[1:]), dtype=ref.dtype, device=ref.device))
    send = torch.cat(pieces) if len(pieces) > 1 else pieces[0]
    M = sum(ms)
    if dist.get_backend(group) == "nccl":
        out = torch.empty((world * M,) + tuple(ref.shape[1:]), dtype=ref.dtype, device=ref.device)
        # RCCL has no int16 type: the same bytes as int32
        dist.all_gather_into_tensor(out.view(torch.int32), send.view(torch.int32), group=group)
        parts = list(out.split(M))
    else:  # gloo (CPU tests): raw bytes
        raw = send.view(torch.uint8)
        parts = [torch.empty_like(raw) for _ in range(world)]
        dist.all_gather(parts, raw, group=group)
        parts = [pp.view(ref.dtype) for pp in parts]
    full, off = [], 0
    for c, m in zip(counts, ms):
        full.append(torch.cat([pp[off:off + cr] for pp, cr in zip(parts, c)]))
        off += m
    return full


def _all_gather_padded(send, m, group):
    """all_gather of equally sized (padded) 1-D/2-D shards; raw bytes over gloo."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if dist.get_backend(group) == "nccl":
        out = torch.empty((world * m,) + tuple(send.shape[1:]), dtype=send.dtype, device=send.device)
        dist.all_gather_into_tensor(out, send, group=group)
        return list(out.split(m))
    raw = send.view(torch.uint8)
    parts = [torch.empty_like(raw) for _ in range(world)]
    dist.all_gather(parts, raw, group=group)
    return [p.view(send.dtype) for p in parts]


def gather_symbols(offsets, symbols, group=None):
    """All-gather every rank's run-length stream (dctq_encode_planes / rle_encode:
    offsets [n_r + 1] int32 holding uint32 bit patterns, symbols [offsets[n_r]] --
    int32 (4-byte symbols) or int16 (the 2-byte format of plans that bound every
    quantized coefficient by 511)) into the stream of the unsharded input on every
    rank: (offsets [N + 1], symbols [total]), rank r's offsets shifted by the
    symbols of ranks < r.

    Two collectives: the per-rank sizes (2 int64), then the padded streams --
    offsets and symbols travel in one byte buffer, so a shard costs 4 B per block
    plus 2 or 4 B per symbol on the wire instead of 128 B per block."""
    import torch
    n = offsets.numel() - 1
    total = int(offsets[n].item()) & 0xFFFFFFFF
    if symbols.numel() < total:
        raise ValueError("symbols shorter than offsets[n]")
    if symbols.dtype not in (torch.int16, torch.int32):
        raise ValueError("symbols must be int16 (2-byte format) or int32 (4-byte format)")
    w = symbols.element_size()
    dev = offsets.device
    sizes = torch.tensor([n, total], dtype=torch.int64, device=dev)
    allsz = _all_gather_padded(sizes.view(1, 2), 1, group)
    ns = [int(t[0, 0]) for t in allsz]
    tots = [int(t[0, 1]) for t in allsz]
    m = max((4 * a + w * b + 3) // 4 * 4 for a, b in zip(ns, tots))
    send = torch.zeros(m, dtype=torch.uint8, device=dev)
    send[:4 * n] = offsets[:n].contiguous().view(torch.uint8)
    send[4 * n:4 * n + w * total] = symbols[:total].contiguous().view(torch.uint8)
    parts = _all_gather_padded(send, m, group)
    offs, syms, base = [], [], 0
    for p, nr, tr in zip(parts, ns, tots):
        offs.append((p[:4 * nr].view(torch.int32).to(torch.int64) & 0xFFFFFFFF) + base)
        syms.append(p[4 * nr:4 * nr + w * tr].view(symbols.dtype))
        base += tr
    offs.append(torch.tensor([base], dtype=torch.int64, device=dev))
    return torch.cat(offs).to(torch.int32), torch.cat(syms)


def max_over_ranks(seconds: float, device, group=None) -> float:
    """Wall time of a timed region as the job sees it: the slowest rank's."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def equals_unsharded(full, chunks) -> bool:
    """Whether a gathered [sum(counts), ...] tensor equals the unsharded result,
    given as `chunks`: an iterable of (first_block, expected) pieces that tile
    the whole output in order (each rank recomputes them locally, so a wrong peer
    offset or rank order that every gather shape shares is caught -- comparing
    the shapes with each other, or a rank's own slice, would not).  Pieces are
    compared as they come, so the full expected tensor never exists at once."""
    import torch
    end = 0
    for first, want in chunks:
        if first != end or first + want.shape[0] > full.shape[0]:
            return False
        if not torch.equal(full[first:first + want.shape[0]], want.to(full.device)):
            return False
        end = first + want.shape[0]
    return end == full.shape[0]


def strong_gather_leg(forward, frames, counts, steps: int, device, sync=lambda: None, group=None,
                      methods=GATHER_METHODS, unsharded=None) -> dict:
    """BASELINE configs[3]: a fixed batch of frames split over the ranks
    (strong scaling; `frames` is this rank's frame_shard), forward DCT+quant of
    the shard, then the coefficient planes gathered onto every rank.

    forward(frames) -> int16 [counts[rank], 64] (the device kernel on the GPU,
    anything equivalent in the CPU tests); `sync` waits for the device.  Timed
    loops of `steps` steps, each bracketed by a barrier and `sync`, the time the
    max over ranks:
      kernel-only : forward alone -> the aggregate rate of the GPUs' kernels;
    and for each gather method (GATHER_METHODS: the all-gather collective and
    the direct peer pushes, SURVEY 8(e)'s two shapes):
      end-to-end  : forward + gather_coefficients -> what a caller that needs
                    every coefficient on every rank gets (xGMI-bound);
      gather-only : gather_coefficients of the shard already computed -> the
                    exchange alone, for its achieved bytes per second per rank.
    Returns the times (the first method's under the plain keys, every method's
    under by_method[m]), the blocks per step and the last gathered tensor of
    each method (full = the first method's).  With `unsharded` (a callable
    returning equals_unsharded's chunks of the unsharded forward, recomputed on
    this rank), every method's gathered tensor is checked against it:
    by_method[m]["gathered_equals_unsharded"]."""
    import time
    import torch.distributed as dist
    total = sum(counts)

    def timed(fn):
        out = fn()
        sync()
        dist.barrier(group=group)
        sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            out = fn()
        sync()
        return max_over_ranks(time.perf_counter() - t0, device, group), out

    for m in methods:
        _check_method(m)
    t_kernel, local = timed(lambda: forward(frames))
    by = {}
    for m in methods:
        t_e2e, full = timed(lambda: gather_coefficients(forward(frames), counts, group, m))
        t_gather, _ = timed(lambda: gather_coefficients(local, counts, group, m))
        by[m] = {"end_to_end_s": t_e2e, "gather_s": t_gather, "full": full}
        if unsharded is not None:
            by[m]["gathered_equals_unsharded"] = equals_unsharded(full, unsharded())
    first = by[methods[0]]
    return {"blocks_per_step": total, "steps": steps, "kernel_s": t_kernel, "end_to_end_s": first["end_to_end_s"],
            "gather_s": first["gather_s"], "local": local, "full": first["full"], "by_method": by}


# xGMI on an MI355X node is point-to-point, 7 links of ~153 GB/s per
# GPU, one to each peer.  A rank of an N-rank gather can take in at most
# (N - 1) x 153 GB/s (every peer pushing over its own link at once); a ring
# that receives over one link per step is held to ~153 GB/s.
XGMI_LINK_GBS = 153.0


def xgmi_report(bytes_received: int, seconds_per_gather: float, world: int) -> dict:
    """Achieved ingress of one rank's gather against the xGMI cost model, so a
    scaling line says which regime its exchange ran in (direct pushes or a
    ring) -- SURVEY 8(e), VERDICT r02 item 7."""
    gbs = bytes_received / seconds_per_gather / 1e9 if seconds_per_gather > 0 else 0.0
    direct = max(world - 1, 1) * XGMI_LINK_GBS
    return {"bytes_received_per_rank": int(bytes_received), "us_per_gather": seconds_per_gather * 1e6,
            "achieved_GBs_per_rank": gbs, "direct_estimate_GBs": direct, "frac_of_direct_estimate": gbs / direct,
            "ring_one_link_estimate_GBs": XGMI_LINK_GBS, "frac_of_ring_estimate": gbs / XGMI_LINK_GBS,
            "model": f"{max(world - 1, 1)} peer links x {XGMI_LINK_GBS:g} GB/s ingress (direct) vs one link (ring)"}
