"""Single-pulse boxcar search over DM-time planes.

The consumer of the sweep's plane: every rank searches the planes it swept
and only candidates (16 B each) leave the GPU, so a DM-sharded or time-block
sharded run never gathers planes.  The reference has no search; its boxcar
is ``Pulse.smooth`` (formats/pulse.py:217-241, tophat ones(w)/sqrt(w), after
PRESTO's single_pulse_search.py).  Definition (pypulsar_amd/csrc/
pdd_search.hip, restated in oracle/search_oracle.py):

* per DM row, chunks of ``detrendlen`` samples are detrended (mean removed)
  and normalised by their own standard deviation;
* boxcar S/N ``snr_w[t] = sum(z[t:t+w]) / sqrt(w)`` for every width of
  ``widths`` and every start ``t <= n - w``;
* one candidate per (DM row, window of 1024 starts): the best (width, start)
  of the window, kept when its S/N >= ``threshold``.

Candidates come back as a NumPy record array with the columns of PRESTO's
``.singlepulse`` files (DM, Sigma, Time, Sample, Downfact) plus the row
index, sorted by (DM row, sample).  No CPU fallback.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import call, ptr, stream_ptr

DEFAULT_WIDTHS = (1, 2, 3, 4, 6, 9, 14, 20, 30, 45, 70, 100, 150)
WINDOW = 1024  # starts per candidate window (kSpWin in pdd_search.hip)
PREFIX_BLOCK = 4096  # starts per k_sp_search block: its prefix sums restart there (kSpStarts)

CAND_DTYPE = np.dtype([("DM", "f8"), ("Sigma", "f4"), ("Time", "f8"), ("Sample", "i8"),
                       ("Downfact", "i4"), ("row", "i4")])


def _widths(widths):
    w = np.ascontiguousarray(np.asarray(widths, dtype=np.int32))
    assert w.ndim == 1 and 1 <= len(w) <= 32, "1..32 boxcar widths"
    assert np.all(w >= 1) and np.all(w <= 1025), "widths must be in 1..1025"
    assert np.all(np.diff(w) > 0), "widths must ascend"
    return w


class SinglePulseSearch(object):
    """``SinglePulseSearch(threshold=6.0)(plane, dms, dt)`` -> candidates.

    ``plane``: [D, n] float32 device tensor (a sweep plane, any row stride);
    ``dms``: the D trial DMs of its rows; ``dt``: its sample time;
    ``t0``: sample index of plane column 0 (e.g. a block's start in a stream);
    ``starttime``: the time of sample 0."""

    def __init__(self, threshold=6.0, widths=DEFAULT_WIDTHS, detrendlen=1000, max_cands=1 << 20):
        _lib.require_gpu()
        self.threshold = float(threshold)
        self.widths = _widths(widths)
        self.detrendlen = int(detrendlen)
        assert self.detrendlen >= 1
        self.max_cands = int(max_cands)

    def stats(self, plane, stream=None):
        """Per-chunk (mean, 1/std) of a [D, n] plane: [D, ceil(n/L)] each."""
        assert plane.is_cuda and plane.dtype == torch.float32 and plane.dim() == 2
        assert plane.stride(1) == 1
        D, n = plane.shape
        nchunk = -(-n // self.detrendlen)
        mean = torch.empty((D, nchunk), dtype=torch.float32, device=plane.device)
        istd = torch.empty_like(mean)
        if D and n:
            call("pdd_sp_chunk_stats", ptr(plane), D, n, plane.stride(0), self.detrendlen,
                 ptr(mean), ptr(istd), stream_ptr(stream))
        return mean, istd

    def raw(self, plane, stream=None, stats=None, nxt=None, n_starts=None):
        """Device-side search; returns (cands int32 [max_cands, 4] = row,
        start, width, snr bits; count tensor) without synchronising.
        ``nxt`` = (next plane, its stats): the rows continue into the next
        plane of a stream (plane width must be a multiple of detrendlen);
        ``n_starts`` limits the searched starts (default: all)."""
        D, n = plane.shape
        dev = plane.device
        mean, istd = self.stats(plane, stream) if stats is None else stats
        cands = torch.empty((self.max_cands, 4), dtype=torch.int32, device=dev)
        count = torch.zeros(1, dtype=torch.int64, device=dev)
        if D == 0 or n == 0:
            return cands[:0], count
        xn, n_next, ldn, mn, sn = None, 0, 0, None, None
        if nxt is not None:
            xn, (mn, sn) = nxt
            assert xn.shape[0] == D and xn.stride(1) == 1
            assert n % self.detrendlen == 0, "a continued plane needs width % detrendlen == 0"
            n_next, ldn = xn.shape[1], xn.stride(0)
            nc = -(-n_next // self.detrendlen)  # the next plane's chunks in use
            mn, sn = mn[:, :nc].contiguous(), sn[:, :nc].contiguous()
        if n_starts is None:
            n_starts = n + n_next
        call("pdd_sp_search", ptr(plane), D, n, plane.stride(0), self.detrendlen, ptr(mean),
             ptr(istd), ptr(xn) if n_next else None, n_next, ldn,
             ptr(mn) if n_next else None, ptr(sn) if n_next else None, n_starts,
             self.widths.ctypes.data_as(ctypes.c_void_p), len(self.widths),
             ctypes.c_float(self.threshold), ptr(cands), self.max_cands, ptr(count),
             stream_ptr(stream))
        return cands, count

    def collect(self, cands, count, dms, dt, t0=0, starttime=0.0):
        """Device (cands, count) -> sorted candidate records (synchronises)."""
        k = int(count.item())
        if k > self.max_cands:
            raise RuntimeError("single-pulse search: %d candidates exceed max_cands=%d "
                               "(raise the threshold or max_cands)" % (k, self.max_cands))
        return to_records(cands[:k].cpu().numpy(), dms, dt, t0, starttime)

    def __call__(self, plane, dms, dt, t0=0, starttime=0.0, stream=None):
        dms = np.atleast_1d(np.asarray(dms, dtype=np.float64))
        assert len(dms) == plane.shape[0], "one DM per plane row"
        cands, count = self.raw(plane, stream)
        return self.collect(cands, count, dms, dt, t0, starttime)


class StreamingSearch(object):
    """Streaming FRB pipeline: ``StreamingSweep`` blocks (zero-DM, downsample,
    DM sweep; BASELINE config 5) searched one block behind the sweep, each
    block's rows continued into the next block's plane, so the candidates
    equal those of a one-shot search of the whole stream's plane.  Needs the
    plane block width (block / downsamp) to be a multiple of the detrend
    length and of the 4096-start search block (k_sp_search's prefix sums
    restart every 4096 starts, so equal S/N bits -- hence equal candidates --
    need the stream's block seams on those boundaries).  Yields candidate
    record arrays.  Preallocated ``planes`` (see StreamingSweep) must number
    at least 2: a block's plane is read again when the next block's plane is
    searched (they rotate by emitted block, so 2 suffice)."""

    def __init__(self, dms, freqs, dt, block=1 << 18, downsamp=2, zero_dm=True, dtype=None,
                 threshold=6.0, widths=DEFAULT_WIDTHS, detrendlen=1024, max_cands=1 << 20):
        from .stream import StreamingSweep
        kw = {} if dtype is None else {"dtype": dtype}
        self.sweep = StreamingSweep(dms, freqs, dt, block=block, downsamp=downsamp,
                                    zero_dm=zero_dm, **kw)
        self.search = SinglePulseSearch(threshold, widths, detrendlen, max_cands)
        nb = self.sweep.n_out_block
        assert nb % detrendlen == 0 and nb % PREFIX_BLOCK == 0, \
            "block/downsamp must be a multiple of detrendlen and of %d" % PREFIX_BLOCK
        self.dms = np.asarray(dms, dtype=np.float64)
        self.dt = dt * downsamp

    def __call__(self, chunks, planes=None, starttime=0.0):
        assert planes is None or len(planes) >= 2
        halo = int(self.search.widths[-1]) - 1
        prev = None  # (t0, plane, stats)
        for t0, plane in self.sweep(chunks, planes):
            st = self.search.stats(plane)
            if prev is not None:
                p0, pp, ps = prev
                h = min(halo, plane.shape[1])
                c, k = self.search.raw(pp, stats=ps, nxt=(plane[:, :h], st) if h else None,
                                       n_starts=pp.shape[1])
                yield self.search.collect(c, k, self.dms, self.dt, p0, starttime)
            prev = (t0, plane, st)
        if prev is not None:
            p0, pp, ps = prev
            c, k = self.search.raw(pp, stats=ps)
            yield self.search.collect(c, k, self.dms, self.dt, p0, starttime)

    def close(self):
        self.sweep.close()


def to_records(c, dms, dt, t0=0, starttime=0.0):
    """int32 [k, 4] (row, start, width, snr bits) -> sorted CAND_DTYPE records."""
    c = np.asarray(c, dtype=np.int32).reshape(-1, 4)
    out = np.empty(len(c), dtype=CAND_DTYPE)
    out["row"] = c[:, 0]
    out["DM"] = np.asarray(dms, dtype=np.float64)[c[:, 0]] if len(c) else []
    out["Sigma"] = c[:, 3].view(np.float32)
    out["Sample"] = c[:, 1].astype(np.int64) + int(t0)
    out["Time"] = starttime + out["Sample"] * dt
    out["Downfact"] = c[:, 2]
    return np.sort(out, order=("row", "Sample"))


def merge(parts):
    """Concatenate candidate arrays from several planes / ranks, sorted by
    (DM, sample)."""
    parts = [p for p in parts if p is not None and len(p)]
    if not parts:
        return np.empty(0, dtype=CAND_DTYPE)
    return np.sort(np.concatenate(parts), order=("DM", "Sample"))


def write_singlepulse(cands, fn):
    """PRESTO ``.singlepulse`` text layout: '# DM Sigma Time (s) Sample Downfact'."""
    with open(fn, "w") as f:
        f.write("# DM      Sigma      Time (s)     Sample    Downfact\n")
        for c in cands:
            f.write("%7.2f %7.2f %13.6f %10d     %3d\n"
                    % (c["DM"], c["Sigma"], c["Time"], c["Sample"], c["Downfact"]))


def read_singlepulse(fn):
    """Inverse of write_singlepulse (row indices are not stored: -1)."""
    rows = [l.split() for l in open(fn) if l.strip() and not l.startswith("#")]
    out = np.empty(len(rows), dtype=CAND_DTYPE)
    for i, r in enumerate(rows):
        out[i] = (float(r[0]), float(r[1]), float(r[2]), int(r[3]), int(r[4]), -1)
    return out
