"""Multi-GPU sharding of the DM sweep (one process per GPU, torch.distributed).

Two partitions:

* **DM sharding** (one block, many GPUs): rank ``src`` holds the filterbank
  block; it is broadcast to every rank over RCCL (xGMI), each rank sweeps a
  contiguous slice of the DM grid balanced by work (``dm_slices``), and the
  DM-time planes are gathered to ``dst``.  The collectives are the real
  exchange steps of this partition: the block in, the planes out.
* **time-block sharding** (independent blocks): rank r sweeps its own range of
  output samples, reading input ``[a, b + max_bin)`` (the overlap equals the
  largest delay), with no collective at all; concatenating the ranks' planes
  equals the one-shot plane.  This is what ``bench.py`` runs by default.

The backend is whatever the process group was initialised with: "nccl"
(RCCL) on the GPU box, "gloo" in the CPU tests, where ``sweep_fn`` is
injected by the test.
"""
import numpy as np
import torch
import torch.distributed as dist


def dm_slices(D, world, work=None):
    """Contiguous [lo, hi) DM index ranges, one per rank, balancing the sum of
    per-trial ``work`` (default 1 each; a DDplan step's trial costs
    1/downsamp, DDplan2b.py:272-273)."""
    w = np.ones(D) if work is None else np.asarray(work, dtype=np.float64)
    assert len(w) == D and world >= 1
    cum = np.concatenate([[0.0], np.cumsum(w)])
    bounds = [0]
    for r in range(1, world):
        bounds.append(int(np.searchsorted(cum, cum[-1] * r / world, side="left")))
    bounds.append(D)
    bounds = np.maximum.accumulate(bounds)
    return [(int(bounds[r]), int(bounds[r + 1])) for r in range(world)]


def timeblock_ranges(n_out, world, max_bin):
    """Per rank: (out_lo, out_hi, in_lo, in_hi) so rank r computes plane
    columns [out_lo, out_hi) from input samples [in_lo, in_hi) with
    in_hi = out_hi + max(0, max_bin) (the overlap)."""
    edges = np.linspace(0, n_out, world + 1).astype(np.int64)
    ov = max(0, int(max_bin))
    return [(int(edges[r]), int(edges[r + 1]), int(edges[r]), int(edges[r + 1]) + ov)
            for r in range(world)]


def broadcast_block(x, src=0, group=None):
    """Send the block held by ``src`` to every rank (RCCL broadcast over xGMI
    on the GPU box).  ``x`` must be allocated with the block's shape/dtype on
    every rank."""
    dist.broadcast(x, src=src, group=group)
    return x


def allgather_block(part, group=None):
    """Assemble a time-major block from per-rank slices: rank r holds spectra
    [r*n, (r+1)*n) ([n, C], e.g. its own H2D of 1/world of the pinned host
    block) and every rank receives the whole [world*n, C] block.  On the GPU
    box this is one RCCL all-gather over the xGMI mesh: each GPU receives
    (world-1)/world of the block over world-1 distinct links at once, where a
    ring broadcast pushes the whole block through every link in turn
    (~14 ms vs ~112 ms for 17 GB at 8 GPUs)."""
    world = dist.get_world_size(group)
    out = torch.empty((part.shape[0] * world,) + tuple(part.shape[1:]), dtype=part.dtype,
                      device=part.device)
    if hasattr(dist, "all_gather_into_tensor") and part.is_cuda:
        dist.all_gather_into_tensor(out, part.contiguous(), group=group)
    else:
        dist.all_gather(list(out.chunk(world)), part.contiguous(), group=group)
    return out


def dm_sharded_sweep_ag(part_tc, dms, freqs, dt, n_out, sweep_fn=None, to_cm=None, work=None,
                        group=None):
    """DM sharding with the all-gather input exchange: every rank contributes
    its slice of the time-major block, all ranks assemble it
    (``allgather_block``), corner-turn it to [C, N] (``to_cm``, default
    pdd_corner_turn) and sweep their own DM slice; the plane stays on the
    rank (returned with the slice) for a downstream search."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    slices = dm_slices(len(dms), world, work)
    blk = allgather_block(part_tc, group=group)
    if to_cm is None:
        from ._lib import call, ptr, stream_ptr
        from . import _lib
        codes = {torch.uint8: _lib.U8, torch.float32: _lib.F32}
        N, C = blk.shape
        x = torch.empty((C, N), dtype=blk.dtype, device=blk.device)
        call("pdd_corner_turn", ptr(blk), codes[blk.dtype], N, C, C, ptr(x), codes[blk.dtype],
             N, stream_ptr())
    else:
        x = to_cm(blk)
    lo, hi = slices[rank]
    if sweep_fn is None:
        from .sweep import DMSweep

        def sweep_fn(b, sub):
            code = "u8" if b.dtype == torch.uint8 else "f32"
            out = torch.empty((len(sub), n_out), dtype=torch.float32, device=b.device)
            DMSweep(sub, freqs, dt, dtype=code)(b, out=out)
            return out
    part = sweep_fn(x, dms[lo:hi])[:, :n_out] if hi > lo else None
    return (lo, hi), part


def gather_planes(plane, slices, dst=0, group=None):
    """Gather per-rank planes (rows = that rank's DM slice) to ``dst``;
    returns the full [D, n_out] plane on dst, None elsewhere.  Planes are
    padded to the largest slice so every rank sends one equal-size tensor."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    rows = max(hi - lo for lo, hi in slices)
    n_out = plane.shape[1]
    buf = torch.zeros((rows, n_out), dtype=plane.dtype, device=plane.device)
    buf[: plane.shape[0]] = plane
    gl = [torch.empty_like(buf) for _ in range(world)] if rank == dst else None
    dist.gather(buf, gather_list=gl, dst=dst, group=group)
    if rank != dst:
        return None
    return torch.cat([gl[r][: hi - lo] for r, (lo, hi) in enumerate(slices)], dim=0)


def dm_sharded_sweep(x, shape, dtype, dms, freqs, dt, n_out, sweep_fn=None, src=0, dst=0,
                     work=None, group=None, device=None):
    """Broadcast one block from ``src``, sweep this rank's DM slice, gather the
    planes to ``dst``.  ``x`` is the block on ``src`` (ignored elsewhere).
    ``sweep_fn(x, dms_slice) -> [len(slice), n_out] plane`` defaults to the
    HIP DMSweep."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    slices = dm_slices(len(dms), world, work)
    if rank != src:
        x = torch.empty(shape, dtype=dtype, device=device)
    broadcast_block(x, src=src, group=group)
    lo, hi = slices[rank]
    if sweep_fn is None:
        from .sweep import DMSweep

        def sweep_fn(blk, sub):
            code = "u8" if blk.dtype == torch.uint8 else "f32"
            sw = DMSweep(sub, freqs, dt, dtype=code)
            out = torch.empty((len(sub), n_out), dtype=torch.float32, device=blk.device)
            sw(blk, out=out)
            return out
    if hi > lo:
        part = sweep_fn(x, dms[lo:hi])[:, :n_out]
    else:
        part = torch.zeros((0, n_out), dtype=torch.float32, device=x.device)
    return gather_planes(part, slices, dst=dst, group=group)


def gather_candidates(cands, group=None):
    """All-gather per-rank candidate record arrays (small: 40 B each) and
    merge them, sorted by (DM, sample), on every rank."""
    from .search import merge
    world = dist.get_world_size(group)
    parts = [None] * world
    dist.all_gather_object(parts, cands, group=group)
    return merge(parts)


def dm_sharded_search(x, shape, dtype, dms, freqs, dt, n_out, sweep_fn=None, search_fn=None,
                      src=0, work=None, group=None, device=None, threshold=6.0):
    """DM sharding with the search on the rank that swept: broadcast one block
    from ``src``, sweep this rank's DM slice, search its plane locally and
    exchange only the candidates -- the DM-time planes never leave their GPU
    ("keep them resident per rank for a downstream search").
    Every DM row is searched whole on one rank, so the merged list equals the
    single-GPU search of the full plane.  ``search_fn(plane, dms_slice) ->
    records`` defaults to the HIP SinglePulseSearch."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    slices = dm_slices(len(dms), world, work)
    if rank != src:
        x = torch.empty(shape, dtype=dtype, device=device)
    broadcast_block(x, src=src, group=group)
    lo, hi = slices[rank]
    if sweep_fn is None:
        from .sweep import DMSweep

        def sweep_fn(blk, sub):
            code = "u8" if blk.dtype == torch.uint8 else "f32"
            sw = DMSweep(sub, freqs, dt, dtype=code)
            out = torch.empty((len(sub), n_out), dtype=torch.float32, device=blk.device)
            sw(blk, out=out)
            return out
    if search_fn is None:
        from .search import SinglePulseSearch
        sps = SinglePulseSearch(threshold=threshold)

        def search_fn(plane, sub):
            return sps(plane, sub, dt)
    cands = None
    if hi > lo:
        cands = search_fn(sweep_fn(x, dms[lo:hi])[:, :n_out], dms[lo:hi])
    return gather_candidates(cands, group=group)
