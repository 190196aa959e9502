"""Streaming FRB-style pipeline (BASELINE.json configs[4]; SURVEY.md §8(d)
config 5): continuous filterbank blocks -> zero-DM -> downsample -> batched DM
sweep, with pinned-host H2D copies overlapped with compute.

Zero-DM modes (bin/zero_dm_filter.py:30-39 subtracts each spectrum's channel
mean; for integer data the mean is rounded half-to-even and the difference is
taken in the data dtype):
  * ``"auto"`` (default): ``"wrap"`` -- the reference's uint8 result --
    where the exact path applies (8-bit input), else ``"float"``.
  * ``"int"`` (8-bit input, downsamp <= 2): x - round(mean) as an
    exact signed integer (the reference's rounding without the uint8 wrap),
    co-added and offset into 16-bit samples <= 1023 (pdd_zdm_int_downsample)
    so the exact packed-u16 sweep runs; the plane bias is removed in the
    sweep epilogue.  Every plane value is an exact integer.
  * ``"wrap"``: the reference's uint8 result, (x - round(mean)) mod 256, on
    the same exact 16-bit path (downsamp <= 4).
  * ``"float"`` (``True``): x - mean in float32, then the float32 sweep
    (the reference's semantics for float data).
  * ``False``: no filter (8-bit input, downsamp <= 4: exact 16-bit path).

Per input chunk (``block`` spectra of the stream, time-major [n, nchan] in
file order, 8/16-bit or float32):

    copy stream : pinned chunk i --H2D--> raw[i % 3][0:ov]      (head, event)
                  pinned chunk i --H2D--> raw[i % 3][ov:n]     (rest, event)
    compute     : raw[(i-1) % 3][block : block + ov] <- raw[i % 3][0 : ov]   (D2D)
                  prologue(raw[(i-1) % 3])  -> [C, (block + ov)/ds] u16 (or f32)
                  DMSweep (interleave + sweep, trim)   -> plane [D, block/ds]

``ov = max_bin * ds`` input spectra (the largest dispersion delay of the grid
at the downsampled rate) of chunk i are appended to block i-1, so the
concatenated per-block planes are exactly -- bit for bit -- the plane of the
one-shot ``zero_dm -> downsample -> sweep(trim=True)`` over the whole stream
(zero-DM is per spectrum, downsampling groups stay aligned because
block % ds == 0, and every plane column sees all of its inputs).

Block i-1 waits only for the HEAD of chunk i (its overlap), so the rest of
chunk i's H2D runs on the copy stream while block i-1 is processed; three raw
buffers rotate so the next chunk's copy never waits for the block being
computed.  Events guard every hand-off.  No CPU fallback.
"""
import numpy as np
import torch

from . import _lib
from ._lib import call, ptr, stream_ptr
from .sweep import DMSweep

_CODES = {torch.uint8: _lib.U8, torch.int16: _lib.U16, torch.float32: _lib.F32}


_ZDM = {"none": _lib.ZDM_NONE, "int": _lib.ZDM_INT, "wrap": _lib.ZDM_WRAP}


def prologue(raw, n, C, ds, mode, img, offset=0, stream=None):
    """zero-DM (``mode``) + downsample by ``ds`` + corner turn of the
    time-major block raw[:n] into the channel-major image ``img``: 16-bit
    offset integers (pdd_zdm_int_downsample) when ``img`` is int16, float32
    (pdd_zdm_downsample) otherwise."""
    if img.dtype == torch.int16:
        call("pdd_zdm_int_downsample", ptr(raw), _lib.U8, n, C, raw.stride(0), ds, _ZDM[mode],
             offset, ptr(img), img.stride(0), stream_ptr(stream))
    else:
        call("pdd_zdm_downsample", ptr(raw), _CODES[raw.dtype], n, C, raw.stride(0), ds,
             int(mode != "none"), ptr(img), img.stride(0), stream_ptr(stream))
    return img


class StreamingSweep(object):
    """``StreamingSweep(dms, freqs, dt)(chunks)`` yields ``(t0, plane)``:
    plane columns t0 .. t0 + plane.shape[1] - 1 of the stream's DM-time plane
    (downsampled time index)."""

    def __init__(self, dms, freqs, dt, block=1 << 18, downsamp=2, zero_dm="auto",
                 dtype=torch.uint8, device="cuda"):
        _lib.require_gpu()
        assert block % downsamp == 0 and 64 % downsamp == 0
        self.freqs = np.asarray(freqs, dtype=np.float64)
        self.C = len(self.freqs)
        self.ds = int(downsamp)
        self.dt = dt
        mode = {True: "float", False: "none"}.get(zero_dm, zero_dm)
        if mode == "auto":
            # the reference's own result for 8-bit data: uint8 wrap
            # (zero_dm_filter.py:30-39), exact on the 16-bit path
            mode = "wrap" if (dtype == torch.uint8 and self.C % 16 == 0 and self.ds <= 4) else "float"
        if mode not in ("int", "wrap", "float", "none"):
            raise ValueError("zero_dm must be 'auto', 'int', 'wrap', 'float', True or False")
        self.dtype = dtype
        self.device = torch.device(device)
        # the exact 16-bit path: 8-bit input, 16-B rows, co-added values <= 1023
        self.exact = (dtype == torch.uint8 and mode != "float" and self.C % 16 == 0
                      and self.ds <= (2 if mode == "int" else 4))
        if mode in ("int", "wrap") and not self.exact:
            raise ValueError("zero_dm=%r needs 8-bit input, nchan %% 16 == 0 and downsamp <= %d"
                             % (mode, 2 if mode == "int" else 4))
        self.mode = mode
        self.zero_dm = mode != "none"
        self.offset = 255 * self.ds if mode == "int" else 0
        # bound of the 16-bit image: offset + co-added (x - round(mean)) for
        # "int" (<= 510 ds), co-added bytes for "wrap" / "none" (<= 255 ds)
        self.input_max = (510 if mode == "int" else 255) * self.ds if self.exact else None
        self.sweep = DMSweep(dms, self.freqs, dt * self.ds, dtype="u16" if self.exact else "f32",
                             input_max=self.input_max)
        self.D = self.sweep.D
        self.max_bin = max(0, self.sweep.max_bin)
        self.block = int(block)
        self.ov = self.max_bin * self.ds
        assert self.ov <= self.block, "block must hold the overlap (max delay x downsamp)"
        n_raw = self.block + self.ov
        self.nbuf = 3
        self.raw = [torch.empty((n_raw, self.C), dtype=dtype, device=self.device)
                    for _ in range(self.nbuf)]
        self.img = torch.empty((self.C, n_raw // self.ds),
                               dtype=torch.int16 if self.exact else torch.float32,
                               device=self.device)
        self.copy_stream = torch.cuda.Stream(device=self.device)
        self.h2d_head = [torch.cuda.Event() for _ in range(self.nbuf)]
        self.h2d = [torch.cuda.Event() for _ in range(self.nbuf)]
        self.free = [torch.cuda.Event() for _ in range(self.nbuf)]
        for e in self.free:
            e.record(torch.cuda.current_stream(self.device))

    @property
    def n_out_block(self):
        return self.block // self.ds

    def _process(self, raw, n_valid, out=None):
        """zero-DM + downsample + sweep of raw[:n_valid] -> plane (trim=True)."""
        nd = n_valid // self.ds
        n_out = max(0, nd - self.max_bin)
        if out is None:
            out = torch.empty((self.D, max(n_out, 0)), dtype=torch.float32, device=self.device)
        if n_out == 0:
            return out[:, :0]
        prologue(raw, n_valid, self.C, self.ds, self.mode, self.img, self.offset)
        self.sweep(self.img[:, :nd], trim=True, out=out, out_bias=-float(self.offset * self.C))
        return out[:, :n_out]

    def __call__(self, chunks, planes=None, start_block=0):
        """chunks: iterable of host tensors [n, C] (pinned for an asynchronous
        copy; every chunk but the last must hold exactly ``block`` spectra).
        planes: optional list of preallocated [D, block/ds] device planes,
        used in rotation by EMITTED-block count (block j -> planes[j % len]),
        so a consumer holding the last len(planes) - 1 planes never sees them
        overwritten.  Yields (t0, plane).

        Restart by block index: a block's plane depends only on its own chunk
        and the head of the next one, so a run resumed at block k -- chunks
        k, k+1, ... of the stream and ``start_block=k`` -- yields exactly the
        (t0, plane) pairs of blocks k, k+1, ... of the uninterrupted run."""
        cur = torch.cuda.current_stream(self.device)
        prev = None  # (buffer index, n spectra)
        t0 = int(start_block) * self.n_out_block
        i = -1
        emitted = 0
        for i, chunk in enumerate(chunks):
            b = i % self.nbuf
            n = chunk.shape[0]
            assert chunk.shape[1] == self.C and n <= self.block
            head = min(self.ov, n)
            self.copy_stream.wait_event(self.free[b])
            with torch.cuda.stream(self.copy_stream):
                if head:
                    self.raw[b][:head].copy_(chunk[:head], non_blocking=True)
                self.h2d_head[b].record(self.copy_stream)
                if n > head:
                    self.raw[b][head:n].copy_(chunk[head:], non_blocking=True)
            self.h2d[b].record(self.copy_stream)
            if prev is not None:
                pb, pn = prev
                assert pn == self.block, "only the last chunk may be short"
                cur.wait_event(self.h2d[pb])       # the block's own chunk
                cur.wait_event(self.h2d_head[b])   # the next chunk's first ov spectra
                if head:
                    self.raw[pb][pn:pn + head].copy_(self.raw[b][:head])
                out = None if planes is None else planes[emitted % len(planes)]
                emitted += 1
                plane = self._process(self.raw[pb], pn + head, out)
                self.free[pb].record(cur)
                yield t0, plane
                t0 += plane.shape[1]
            prev = (b, n)
        if prev is not None:
            pb, pn = prev
            cur.wait_event(self.h2d[pb])
            out = None if planes is None else planes[emitted % len(planes)]
            plane = self._process(self.raw[pb], pn, out)
            self.free[pb].record(cur)
            yield t0, plane

    def close(self):
        self.sweep.close()
