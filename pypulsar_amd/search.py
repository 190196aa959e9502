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

    def raw(self, plane, stream=None):
        """Device-side search; returns (cands int32 [k, 4] = row, start, width,
        snr bits, count tensor) without synchronising."""
        assert plane.is_cuda and plane.dtype == torch.float32 and plane.dim() == 2
        assert plane.stride(1) == 1
        D, n = plane.shape
        dev = plane.device
        nchunk = -(-n // self.detrendlen)
        mean = torch.empty((D, nchunk), dtype=torch.float32, device=dev)
        istd = torch.empty_like(mean)
        cands = torch.empty((self.max_cands, 4), dtype=torch.int32, device=dev)
        count = torch.zeros(1, dtype=torch.int64, device=dev)
        if D == 0 or n == 0:
            return cands[:0], count
        s = stream_ptr(stream)
        call("pdd_sp_chunk_stats", ptr(plane), D, n, plane.stride(0), self.detrendlen, ptr(mean),
             ptr(istd), s)
        call("pdd_sp_search", ptr(plane), D, n, plane.stride(0), self.detrendlen, ptr(mean),
             ptr(istd), self.widths.ctypes.data_as(ctypes.c_void_p), len(self.widths),
             ctypes.c_float(self.threshold), ptr(cands), self.max_cands, ptr(count), s)
        return cands, count

    def __call__(self, plane, dms, dt, t0=0, starttime=0.0, stream=None):
        dms = np.atleast_1d(np.asarray(dms, dtype=np.float64))
        assert len(dms) == plane.shape[0], "one DM per plane row"
        cands, count = self.raw(plane, stream)
        k = int(count.item())
        if k > self.max_cands:
            raise RuntimeError("single-pulse search: %d candidates exceed max_cands=%d "
                               "(raise the threshold or max_cands)" % (k, self.max_cands))
        c = cands[:k].cpu().numpy()
        return to_records(c, dms, dt, t0, starttime)


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
