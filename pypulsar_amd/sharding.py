"""Multi-GPU sharding of the DM sweep (one process per GPU, torch.distributed).

Two partitions:

* **DM sharding** (one block, many GPUs; the north star and BASELINE
  configs[3]): every GPU needs the whole filterbank block and owns a
  contiguous slice of the DM grid, balanced by DDplan work fraction
  (``dm_slices``; DDplan2b.py:272-273).  ``DMShardedSweep`` is the pipelined
  production path: the block enters as per-rank H2D slices assembled by RCCL
  all-gathers over xGMI, one time batch at a time, and batch k+1's all-gather
  runs on the communicator's stream while batch k is corner-turned and swept;
  planes stay resident on their rank (or, with ``gather=True``, each batch's
  rows are sent to ``dst`` while the next batch is swept).  The collectives
  are the real exchange steps of this partition: the block in, the planes out.
* **time-block sharding** (independent blocks): rank r sweeps its own range of
  output samples, reading input ``[a, b + max_bin)`` (the overlap equals the
  largest delay), with no collective at all; concatenating the ranks' planes
  equals the one-shot plane.

The backend is whatever the process group was initialised with: "nccl"
(RCCL) on the GPU box, "gloo" in the CPU tests, where the per-rank compute
(``to_cm``, ``sweep_fn``) is injected by the test.
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


def trial_work(dms, downsamp=1):
    """Per-trial work weights of a DM grid: DDplan2b's work fraction is
    numDMs/downsamp per step (DDplan2b.py:272-273), i.e. 1/downsamp per
    trial.  ``downsamp`` may be a scalar or one value per trial."""
    d = np.broadcast_to(np.asarray(downsamp, dtype=np.float64), (len(dms),))
    return 1.0 / d


def plan_trial_work(ddplan):
    """(dms, work) over all steps of a DDplan (concatenated in step order)."""
    dms = np.concatenate([np.asarray(s.DMs, dtype=np.float64) for s in ddplan.DDsteps])
    work = np.concatenate([trial_work(s.DMs, s.downsamp) for s in ddplan.DDsteps])
    return dms, work


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


def _all_gather_into(out, part, group=None, async_op=False):
    """out[r*n:(r+1)*n] = rank r's ``part`` (RCCL all-gather on the GPU box;
    per-rank views on gloo)."""
    world = dist.get_world_size(group)
    if part.is_cuda and hasattr(dist, "all_gather_into_tensor"):
        return dist.all_gather_into_tensor(out, part, group=group, async_op=async_op)
    return dist.all_gather(list(out.chunk(world)), part, group=group, async_op=async_op)


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
    _all_gather_into(out, part.contiguous(), group=group)
    return out


def _codes():
    from . import _lib
    return {torch.uint8: _lib.U8, torch.float32: _lib.F32}


def _corner_turn(src_tc, dst_cm):
    """pdd_corner_turn of a time-major [n, C] block into the channel-major
    [C, n] view ``dst_cm`` (row stride = the full block's length)."""
    from ._lib import call, ptr, stream_ptr
    n, C = src_tc.shape
    code = _codes()[src_tc.dtype]
    call("pdd_corner_turn", ptr(src_tc), code, n, C, src_tc.stride(0), ptr(dst_cm), code,
         dst_cm.stride(0), stream_ptr())


class DMShardedSweep(object):
    """Pipelined DM-sharded sweep of ONE filterbank block across the ranks
    (north star; BASELINE configs[3]).

    Semantics: rank r produces rows [lo_r, hi_r) of the one-shot plane
    ``plane[d][t] = sum_c X(c, t + bins[d][c])``, t < n_out = N - max bin of
    the WHOLE grid (per DM trial: Spectra.dedisperse(dms[d], trim=True) +
    channel sum, formats/spectra.py:229-260 + bin/waterfaller.py:140),
    delivered as ``n_batches`` column blocks ``planes[k]`` ([rows, cols_k],
    columns [col_edges[k], col_edges[k+1])).

    Input layout (file order, time-major): the block is cut into ``n_batches``
    time batches of T = N / n_batches spectra; rank r holds, for each batch k,
    spectra [k*T + r*P, k*T + (r+1)*P), P = T/W -- ``part`` is
    [n_batches, P, C] (its own 1/W H2D slice of every batch).

    One ``__call__`` (a bench step), when P is a power of two ("pieces"):
        for k in 0..n_batches-1:
            corner-turn this rank's slice of batch k -> [C, P]   (pdd_corner_turn,
              1/W of the block per rank, not the whole block)
            all-gather batch k's slices (async RCCL) -> pieces [kW, (k+1)W)
              of the [N/P][C][P] block (issued before batch k-1's sweep, so
              the exchange of batch k overlaps the sweep of batch k-1)
            sweep plane columns of batch k-1 straight from the pieces
              (pdd_sweep_execute_ex: pieces layout + column offset)
        (gather=True: each batch's rows are also sent to ``dst``, async,
         which receives them into its full [D, cols_k] batch plane)
    Otherwise the slices are all-gathered time-major and every rank
    corner-turns the whole batch (the same pipeline).  Column block k needs
    input up to col_edges[k+1] + max_bin <= (k+1)T.  All delays are >= 0
    (cur_dm = 0, dms >= 0, reference = the highest frequency), so no pad is
    ever read.

    Plans (delay table, sweep plan, buffers) are built once in __init__;
    ``work`` (per-trial weights, e.g. ``trial_work``) balances the DM slices.
    ``to_cm(src_tc, dst_cm_view)`` and ``sweep_fn(x, N, piece, x_off,
    dms_slice, out, n_cols)`` (piece 0: x channel-major [C, N]) are injected
    by the CPU tests; the defaults are pdd_corner_turn and the HIP DMSweep of
    this rank's slice (built once).

    ``gather_fn(out, cm, k)`` (pieces layout) replaces the async RCCL
    all-gather of batch k -- ``out`` = the batch's [W*C, P] pieces, ``cm`` =
    this rank's corner-turned slice -- and returns an object with ``wait()``
    (the GPU test injects a delayed loopback on a side stream to check the
    pipeline's stream ordering with real HIP kernels).

    Rehearsal (``world=W, rank=r`` given; no process group needed): the
    exact compute of rank r of a W-rank run -- its own slice's corner turn
    into the block, its DM slice swept at the global width, batch by batch
    -- on one device, with the exchange replaced by a block that already
    holds every rank's slices (``prefill`` once, or a shared ``x_buf``).
    Stacking the W ranks' planes gives the one-shot plane; timing each rank
    gives the compute side of the W-GPU step (``bench.py --rehearse W``).
    """

    def __init__(self, dms, freqs, dt, N, dtype=torch.uint8, n_batches=1, work=None,
                 gather=False, dst=0, group=None, device=None, to_cm=None, sweep_fn=None,
                 pieces=None, world=None, rank=None, x_buf=None, gather_fn=None, factor=True):
        from . import delays as _delays
        self.group = group
        self.rehearse = world is not None
        if self.rehearse:
            self.world, self.rank = int(world), int(rank)
            assert 0 <= self.rank < self.world, "rank outside the rehearsed world"
            assert not gather, "a rehearsal has no plane gather (one device)"
        else:
            self.world = dist.get_world_size(group) if dist.is_initialized() else 1
            self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.dms = np.asarray(dms, dtype=np.float64)
        self.freqs = np.asarray(freqs, dtype=np.float64)
        self.C = len(self.freqs)
        self.N = int(N)
        self.D = len(self.dms)
        self.dt = dt
        self.dtype = dtype
        self.device = torch.device("cpu") if device is None else torch.device(device)
        self.nb = int(n_batches)
        assert self.N % (self.nb * self.world) == 0, \
            "N must split into n_batches x world equal slices"
        self.T = self.N // self.nb
        self.P = self.T // self.world
        pow2 = self.P & (self.P - 1) == 0
        self.pieces = pow2 if pieces is None else bool(pieces)
        assert pow2 or not self.pieces, "the pieces layout needs a power-of-two slice length"
        tab = _delays.sweep_table(self.dms, self.freqs, dt)
        assert tab.size == 0 or tab.min() >= 0, "DM-sharded sweep expects delays >= 0"
        self.max_bin = int(tab.max()) if tab.size else 0
        self.n_out = self.N - self.max_bin
        assert self.n_out > 0 and self.T > self.max_bin, \
            "each time batch must be longer than the largest delay"
        edges = [0]
        for k in range(self.nb):
            edges.append(min(self.n_out, (k + 1) * self.T - self.max_bin))
        edges[-1] = self.n_out
        self.col_edges = edges
        self.slices = dm_slices(self.D, self.world, work)
        self.lo, self.hi = self.slices[self.rank]
        self.rows = self.hi - self.lo
        self.gather = bool(gather)
        self.dst = dst
        # buffers (reused every call)
        xshape = (self.N // self.P, self.C, self.P) if self.pieces else (self.C, self.N)
        if x_buf is not None:
            assert tuple(x_buf.shape) == xshape and x_buf.dtype == dtype and x_buf.is_contiguous()
            self.x = x_buf
        else:
            self.x = torch.empty(xshape, dtype=dtype, device=self.device)
        self.gather_fn = gather_fn
        assert gather_fn is None or self.pieces, "gather_fn takes the pieces layout"
        self.direct = self.rehearse and gather_fn is None  # rehearsal writes its piece in place
        if self.pieces:
            # two corner-turn buffers: batch k+1's turn must not overwrite the
            # one batch k's all-gather may still be reading
            self.cm = ([] if self.direct else
                       [torch.empty((self.C, self.P), dtype=dtype, device=self.device)
                        for _ in range(2)])
            self.xt = None
        else:
            self.xt = (torch.empty((self.N, self.C), dtype=dtype, device=self.device)
                       if self.world > 1 and not self.rehearse else None)
        cols = [edges[k + 1] - edges[k] for k in range(self.nb)]
        if self.gather and self.rank == self.dst:
            # dst's full batch planes; its own rows are views of them
            self.full = [torch.empty((self.D, c), dtype=torch.float32, device=self.device)
                         for c in cols]
            self.planes = [f[self.lo:self.hi] for f in self.full]
        else:
            self.full = None
            self.planes = [torch.empty((self.rows, c), dtype=torch.float32, device=self.device)
                           for c in cols]
        self.to_cm = to_cm if to_cm is not None else _corner_turn
        self.sw = None
        if sweep_fn is None:
            from .sweep import DMSweep
            code = "u8" if dtype == torch.uint8 else "f32"
            if self.rows:
                self.sw = DMSweep(self.dms[self.lo:self.hi], self.freqs, dt, dtype=code,
                                  factor=factor)

            def sweep_fn(x, N, piece, x_off, dms_slice, out, n_cols):
                if piece:
                    self.sw.sweep_pieces(x, N, piece, x_off, n_cols, out)
                else:
                    self.sw(x[:, x_off:x_off + n_cols + self.max_bin], out=out, n_out=n_cols)
        self.sweep_fn = sweep_fn

    def __call__(self, part):
        """Run one pipelined sweep of the block whose per-rank slices are
        ``part`` ([n_batches, P, C]).  Returns this rank's batch planes
        (with ``gather``: the full [D, cols_k] batch planes on ``dst``)."""
        nb = self.nb
        assert tuple(part.shape) == (nb, self.P, self.C) and part.dtype == self.dtype
        sends = []
        pending = [None] * nb
        for k in range(nb):
            pending[k] = self.exchange_batch(part, k)  # overlaps batch k-1's sweep
            if k > 0:
                if pending[k - 1] is not None:
                    pending[k - 1].wait()
                sends.extend(self.sweep_batch(k - 1))
        if pending[nb - 1] is not None:
            pending[nb - 1].wait()
        sends.extend(self.sweep_batch(nb - 1))
        for w in sends:
            w.wait()
        return self.full if (self.gather and self.rank == self.dst) else self.planes

    def exchange_batch(self, part, k):
        """Batch k into x: this rank's corner turn (+ the async all-gather of
        every rank's slice); returns the pending collective or None."""
        W, T, P = self.world, self.T, self.P
        if self.direct:
            # this rank's own slice only; the others' are already in x
            r = self.rank
            if self.pieces:
                self.to_cm(part[k], self.x[k * W + r])
            else:
                self.to_cm(part[k], self.x[:, k * T + r * P:k * T + (r + 1) * P])
            return None
        if self.pieces:
            dst = self.x[k * W:(k + 1) * W]  # [W, C, P]
            if W == 1:
                self.to_cm(part[k], dst[0])
                return None
            cm = self.cm[k % 2]
            self.to_cm(part[k], cm)
            if self.gather_fn is not None:
                return self.gather_fn(dst.view(W * self.C, P), cm, k)
            return _all_gather_into(dst.view(W * self.C, P), cm, group=self.group,
                                    async_op=True)
        if W == 1:
            self.to_cm(part[k], self.x[:, k * T:(k + 1) * T])
            return None
        return _all_gather_into(self.xt[k * T:(k + 1) * T], part[k], group=self.group,
                                async_op=True)

    def sweep_batch(self, k):
        """Sweep plane columns of batch k (its exchange complete); returns the
        pending plane sends (``gather``)."""
        W, T = self.world, self.T
        if not self.pieces and W > 1 and not self.rehearse:
            self.to_cm(self.xt[k * T:(k + 1) * T], self.x[:, k * T:(k + 1) * T])
        a, b = self.col_edges[k], self.col_edges[k + 1]
        if self.rows and b > a:
            self.sweep_fn(self.x, self.N, self.P if self.pieces else 0, a,
                          self.dms[self.lo:self.hi], self.planes[k], b - a)
        return self._gather_batch(k) if self.gather else []

    def prefill(self, block_tc):
        """Rehearsal: write the WHOLE time-major [N, C] block into x, as the
        all-gathers of every rank would (once, outside any timing)."""
        assert tuple(block_tc.shape) == (self.N, self.C) and block_tc.dtype == self.dtype
        if self.pieces:
            for b in range(self.N // self.P):
                self.to_cm(block_tc[b * self.P:(b + 1) * self.P], self.x[b])
        else:
            self.to_cm(block_tc, self.x)

    def _gather_batch(self, k):
        """Rows of batch k to ``dst`` (point-to-point, async): dst receives each
        rank's rows straight into its full batch plane (contiguous row range),
        no concatenation."""
        if self.world == 1:
            return []
        if self.rank != self.dst:
            return [dist.isend(self.planes[k], self.dst, group=self.group)] if self.rows else []
        works = []
        for r, (lo, hi) in enumerate(self.slices):
            if r != self.dst and hi > lo:
                works.append(dist.irecv(self.full[k][lo:hi], r, group=self.group))
        return works

    def plane(self):
        """This rank's rows (or dst's full plane with ``gather``) as one
        [rows, n_out] tensor (a copy; for tests and downstream consumers that
        want a single plane -- not used in the timed path)."""
        src = self.full if (self.gather and self.rank == self.dst) else self.planes
        return torch.cat(list(src), dim=1)

    def close(self):
        """Releases the plan and drops the device buffers (planes a caller
        still holds stay valid).  The sweep closure refers back to this
        object, so without close() the buffers live until a garbage
        collection."""
        if self.sw is not None:
            self.sw.close()
            self.sw = None
        self.sweep_fn = None
        self.x = self.full = self.planes = None


def timeshard_edges(n_out, world, align=1024):
    """Plane column edges of a time-sharded sweep: ``world`` ranges of
    (nearly) equal width, interior edges on multiples of ``align`` (the
    sweep's time tile: 1024 samples for both the u16-eighths and the float32
    quarters tiling), so no rank sweeps a partial tile except the last."""
    edges = [0]
    for r in range(1, world):
        e = int(round(n_out * r / world / align)) * align
        edges.append(min(max(e, edges[-1]), n_out))
    edges.append(int(n_out))
    return edges


class TimeShardedSweep(object):
    """Time-sharded sweep of ONE filterbank block across the ranks (SURVEY.md
    §8(e) 2, strong scaling: the block and the grid are fixed, each of W
    GPUs owns a contiguous range of plane COLUMNS and sweeps the whole DM
    grid over it).  No collective: rank r reads input spectra
    [a_r, b_r + max_bin) -- its columns plus an overlap of the largest delay
    (14 504 samples at configs[3], 2.8% of 2^22 / 8) -- straight from the
    file / host (its own H2D), corner-turns them and sweeps columns
    [a_r, b_r) of the one-shot plane
        plane[d][t] = sum_c X(c, t + bins[d][c]),  t < n_out = N - max bin
    (Spectra.dedisperse(dms[d], trim=True) + channel sum, formats/spectra.py
    :229-260 + bin/waterfaller.py:140).  Every trial's delays are >= 0 and
    t + bins <= b_r - 1 + max_bin < in_hi, so no pad is read and the ranks'
    column blocks concatenate to the one-shot plane bit for bit.

    Why a second partition: the exact factorised sweep pays a
    stage 1 per pattern over the whole time range; under DM sharding a rank's
    trial slice still uses about a third of the grid's patterns at W = 8, so
    stage 1 does not shrink with W.  Time sharding keeps every rank's work
    exactly 1/W of the one-GPU step plus the overlap.

    ``part``: this rank's [n_in, C] time-major input (file order).  Planes
    stay resident; ``gather=True`` sends each rank's [D, cols] block to
    ``dst``, which places it in its full [D, n_out] plane.  ``world, rank``
    without a process group: the rehearsal (the rank's compute is the same,
    there is nothing to replace).  ``to_cm`` / ``sweep_fn(x, out, n_cols)``
    are injected by the CPU tests."""

    def __init__(self, dms, freqs, dt, N, dtype=torch.uint8, world=None, rank=None, gather=False,
                 dst=0, group=None, device=None, to_cm=None, sweep_fn=None, factor=True,
                 align=1024):
        from . import delays as _delays
        self.group = group
        if world is not None:
            self.world, self.rank = int(world), int(rank)
            assert 0 <= self.rank < self.world
            assert not gather, "a rehearsal has no plane gather (one device)"
        else:
            self.world = dist.get_world_size(group) if dist.is_initialized() else 1
            self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.dms = np.asarray(dms, dtype=np.float64)
        self.freqs = np.asarray(freqs, dtype=np.float64)
        self.C, self.N, self.D = len(self.freqs), int(N), len(self.dms)
        self.dt, self.dtype = dt, dtype
        self.device = torch.device("cpu") if device is None else torch.device(device)
        tab = _delays.sweep_table(self.dms, self.freqs, dt)
        assert tab.size == 0 or tab.min() >= 0, "time-sharded sweep expects delays >= 0"
        self.max_bin = int(tab.max()) if tab.size else 0
        self.n_out = self.N - self.max_bin
        assert self.n_out > 0
        self.align = int(align)
        self.edges = timeshard_edges(self.n_out, self.world, align)
        self.a, self.b = self.edges[self.rank], self.edges[self.rank + 1]
        self.cols = self.b - self.a
        self.in_lo, self.in_hi = self.a, self.b + self.max_bin   # input spectra of this rank
        self.n_in = self.in_hi - self.in_lo
        self.gather, self.dst = bool(gather), dst
        self.x = torch.empty((self.C, self.n_in), dtype=dtype, device=self.device)
        self.full = None
        if self.gather and self.rank == self.dst:
            self.full = torch.empty((self.D, self.n_out), dtype=torch.float32, device=self.device)
            self.recv = {r: torch.empty((self.D, self.edges[r + 1] - self.edges[r]),
                                        dtype=torch.float32, device=self.device)
                         for r in range(self.world) if r != self.dst}
        self.out = torch.empty((self.D, self.cols), dtype=torch.float32, device=self.device)
        self.to_cm = to_cm if to_cm is not None else _corner_turn
        self.sw = None
        if sweep_fn is None:
            from .sweep import DMSweep
            self.sw = DMSweep(self.dms, self.freqs, dt,
                              dtype="u8" if dtype == torch.uint8 else "f32", factor=factor)

            def sweep_fn(x, out, n_cols):
                self.sw(x, out=out, n_out=n_cols)
        self.sweep_fn = sweep_fn

    def input_range(self, rank=None):
        """[lo, hi) input spectra of ``rank`` (default this rank)."""
        r = self.rank if rank is None else rank
        return self.edges[r], self.edges[r + 1] + self.max_bin

    def __call__(self, part):
        """One step: corner turn of this rank's [n_in, C] spectra, sweep of
        its columns (and, with ``gather``, the blocks to ``dst``).  Returns
        this rank's [D, cols] plane (``dst`` with gather: the full plane)."""
        assert tuple(part.shape) == (self.n_in, self.C) and part.dtype == self.dtype
        self.to_cm(part, self.x)
        if self.cols:
            self.sweep_fn(self.x, self.out, self.cols)
        return self._gathered()

    def _gathered(self):
        """This rank's plane, or (``gather``) the column blocks sent to
        ``dst`` point-to-point: ``dst`` returns the full plane."""
        if not self.gather or self.world == 1:
            return self.out
        if self.rank != self.dst:
            if self.cols:
                dist.send(self.out, self.dst, group=self.group)
            return self.out
        works = [(r, dist.irecv(buf, r, group=self.group)) for r, buf in self.recv.items()
                 if buf.shape[1]]
        self.full[:, self.a:self.b] = self.out
        for r, w in works:
            w.wait()
            self.full[:, self.edges[r]:self.edges[r + 1]] = self.recv[r]
        return self.full

    def host_step(self, hpart, n_batches=4, copy_stream=None):
        """The same step from this rank's input in PINNED HOST memory (the
        PCIe-inclusive form; the filterbank reader fills such
        a buffer, formats/filterbank.py:143-157): the [n_in, C] spectra are
        copied H2D in ``n_batches`` chunks on a copy stream, and the plane
        columns are swept in ``n_batches`` ranges (edges on the 1024-sample
        tile), range k as soon as the chunks holding its input -- its columns
        plus the max-delay overlap -- have landed: chunk k+1's copy runs
        under range k's corner turn and sweep, only chunk 0's is exposed.
        The plane equals __call__'s bit for bit (every range reads only
        in-range samples).  Returns this rank's [D, cols] plane (``dst`` with
        ``gather``: the full plane, as __call__)."""
        assert tuple(hpart.shape) == (self.n_in, self.C) and hpart.dtype == self.dtype
        nb = max(1, min(int(n_batches), max(1, self.cols // self.align)))
        ce = timeshard_edges(self.cols, nb, self.align)            # column ranges (relative)
        # chunk edges rounded up to 16 spectra (capped at n_in): every chunk's
        # corner turn starts on a 16-byte boundary and takes the 16-byte 8-bit
        # path (pdd_corner_turn); a chunk only has to cover its range's input
        ie = [0] + [min(self.n_in, -(-(ce[k + 1] + self.max_bin) // 16) * 16)
                    for k in range(nb - 1)] + [self.n_in]
        if getattr(self, "hx", None) is None:
            self.hx = torch.empty((self.n_in, self.C), dtype=self.dtype, device=self.device)
        if self.device.type != "cuda":
            # (host-only test harness: the same ranges, copies in order)
            for k in range(nb):
                self.hx[ie[k]:ie[k + 1]].copy_(hpart[ie[k]:ie[k + 1]])
                if ie[k + 1] > ie[k]:
                    self.to_cm(self.hx[ie[k]:ie[k + 1]], self.x[:, ie[k]:ie[k + 1]])
                a, b = ce[k], ce[k + 1]
                if b > a:
                    self.sweep_fn(self.x[:, a:b + self.max_bin], self.out[:, a:b], b - a)
            return self._gathered()
        cur = torch.cuda.current_stream(self.device)
        if copy_stream is None:
            # one copy stream per object, created once: streams created per
            # call end up sharing a hardware queue with the compute stream,
            # and the chunk copies then serialise behind the sweeps
            if getattr(self, "_copy_stream", None) is None:
                self._copy_stream = torch.cuda.Stream(device=self.device)
            copy_stream = self._copy_stream
        cs = copy_stream
        landed = [torch.cuda.Event() for _ in range(nb)]
        cs.wait_stream(cur)  # the previous step's reads of hx / x are done
        with torch.cuda.stream(cs):
            for k in range(nb):
                if ie[k + 1] > ie[k]:
                    self.hx[ie[k]:ie[k + 1]].copy_(hpart[ie[k]:ie[k + 1]], non_blocking=True)
                landed[k].record(cs)
        for k in range(nb):
            cur.wait_event(landed[k])
            if ie[k + 1] > ie[k]:
                self.to_cm(self.hx[ie[k]:ie[k + 1]], self.x[:, ie[k]:ie[k + 1]])
            a, b = ce[k], ce[k + 1]
            if b > a:
                self.sweep_fn(self.x[:, a:b + self.max_bin], self.out[:, a:b], b - a)
        return self._gathered()

    def close(self):
        """Releases the plan and drops the device buffers (see
        DMShardedSweep.close)."""
        if self.sw is not None:
            self.sw.close()
            self.sw = None
        self.sweep_fn = None
        self.hx = self.x = self.out = self.full = None
        self.recv = {}


def split_block(block_tc, n_batches, world, rank):
    """This rank's ``part`` of a time-major [N, C] block for DMShardedSweep:
    [n_batches, N/(n_batches*world), C] (a copy)."""
    N, C = block_tc.shape
    T = N // n_batches
    n = T // world
    v = block_tc.reshape(n_batches, world, n, C)
    return v[:, rank].contiguous()


def gather_planes(plane, slices, dst=0, group=None, out=None):
    """Gather per-rank planes (rows = that rank's DM slice) to ``dst`` into
    the preallocated [D, n_out] ``out`` (allocated if None): dst receives each
    rank's rows straight into its row range (point-to-point), no padding and
    no concatenation.  Returns ``out`` on dst, None elsewhere."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if rank != dst:
        if plane.shape[0]:
            dist.send(plane.contiguous(), dst, group=group)
        return None
    D = slices[-1][1]
    if out is None:
        out = torch.empty((D, plane.shape[1]), dtype=plane.dtype, device=plane.device)
    lo, hi = slices[dst]
    out[lo:hi] = plane
    works = []
    for r in range(world):
        lo, hi = slices[r]
        if r != dst and hi > lo:
            works.append(dist.irecv(out[lo:hi], r, group=group))
    for w in works:
        w.wait()
    return out


def _default_sweep_fn(freqs, dt, n_out):
    """HIP DMSweep of a DM slice at the GLOBAL plane width ``n_out``."""
    from .sweep import DMSweep

    def fn(blk, sub):
        code = "u8" if blk.dtype == torch.uint8 else "f32"
        sw = DMSweep(sub, freqs, dt, dtype=code)
        out = torch.empty((len(sub), n_out), dtype=torch.float32, device=blk.device)
        sw(blk, out=out, n_out=n_out)
        sw.close()
        return out
    return fn


def dm_sharded_sweep(x, shape, dtype, dms, freqs, dt, n_out, sweep_fn=None, src=0, dst=0,
                     work=None, group=None, device=None):
    """Broadcast one block from ``src``, sweep this rank's DM slice, gather the
    planes to ``dst`` (the simple, unpipelined form of DMShardedSweep).
    ``x`` is the [C, N] block on ``src`` (ignored elsewhere).
    ``sweep_fn(x, dms_slice) -> [len(slice), n_out] plane`` defaults to the
    HIP DMSweep at the global width ``n_out``."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    slices = dm_slices(len(dms), world, work)
    if rank != src:
        x = torch.empty(shape, dtype=dtype, device=device)
    broadcast_block(x, src=src, group=group)
    lo, hi = slices[rank]
    if sweep_fn is None:
        sweep_fn = _default_sweep_fn(freqs, dt, n_out)
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
        sweep_fn = _default_sweep_fn(freqs, dt, n_out)
    if search_fn is None:
        from .search import SinglePulseSearch
        sps = SinglePulseSearch(threshold=threshold)

        def search_fn(plane, sub):
            return sps(plane, sub, dt)
    cands = None
    if hi > lo:
        cands = search_fn(sweep_fn(x, dms[lo:hi])[:, :n_out], dms[lo:hi])
    return gather_candidates(cands, group=group)
