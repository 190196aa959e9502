"""PRESTO rfifind ``.mask`` files, as bin/waterfaller.py:28-48,92-99 uses them.

The reference imports PRESTO's ``rfifind`` module (not vendored, not
installed here) only for ``rfifind.rfifind(maskfile)`` and two attributes of
the result: ``ptsperint`` and ``mask_zap_chans_per_int``.  This module
restates PRESTO's published ``.mask`` layout (little-endian, as rfifind's C
writer emits it on x86):

    float64 x 6  time_sig, freq_sig, MJD, dtint, lofreq, df
    int32 x 3    nchan, nint, ptsperint
    int32        nzap_chans, then that many channel numbers      (zapped everywhere)
    int32        nzap_ints,  then that many interval numbers     (zapped entirely)
    int32 x nint zapped-channel count of every interval, then for every
                 interval with 0 < count < nchan, its channel numbers
                 (count == nchan means every channel, stored without a list)

Parity with PRESTO itself is UNPINNED (PRESTO is absent and the reference
ships no mask file): tested by write -> read round trips and by the
waterfaller ``--mask`` path against the oracle's masked().
"""
import numpy as np


class rfifind(object):
    """``rfifind(filename)``: the mask of an rfifind run (attribute names as
    PRESTO's rfifind.rfifind)."""

    def __init__(self, filename):
        self.basename = filename[:filename.rfind("_rfifind.")] if "_rfifind." in filename \
            else filename
        self.read_mask(filename)

    def read_mask(self, filename):
        with open(filename, "rb") as f:
            buf = f.read()
        pos = [0]

        def take(dtype, count):
            dt = np.dtype(dtype).newbyteorder("<")
            n = dt.itemsize * count
            if pos[0] + n > len(buf):
                raise ValueError("%s: truncated rfifind mask" % filename)
            a = np.frombuffer(buf, dtype=dt, count=count, offset=pos[0])
            pos[0] += n
            return a.astype(dt.newbyteorder("="))

        (self.time_sig, self.freq_sig, self.MJD, self.dtint, self.lofreq,
         self.df) = (float(v) for v in take(np.float64, 6))
        self.nchan, self.nint, self.ptsperint = (int(v) for v in take(np.int32, 3))
        if self.nchan <= 0 or self.nint < 0 or self.ptsperint <= 0:
            raise ValueError("%s: bad rfifind mask header" % filename)
        self.freqs = self.lofreq + np.arange(self.nchan) * self.df
        self.times = np.arange(self.nint) * self.dtint
        nz = int(take(np.int32, 1)[0])
        self.mask_zap_chans = set(int(c) for c in take(np.int32, nz))
        nz = int(take(np.int32, 1)[0])
        self.mask_zap_ints = take(np.int32, nz)
        counts = take(np.int32, self.nint)
        self.mask_zap_chans_per_int = []
        for n in counts:
            if n == self.nchan:
                z = np.arange(self.nchan, dtype=np.int32)
            elif n > 0:
                z = take(np.int32, int(n))
            else:
                z = np.zeros(0, dtype=np.int32)
            self.mask_zap_chans_per_int.append(z)


def write_mask(filename, nchan, ptsperint, zap_chans_per_int, zap_chans=(), zap_ints=(),
               time_sig=10.0, freq_sig=4.0, mjd=0.0, dtint=1.0, lofreq=1250.0, df=1.0):
    """Write a ``.mask`` file in the layout above (for tests and tools)."""
    per = [np.asarray(z, dtype=np.int32).ravel() for z in zap_chans_per_int]
    parts = [np.array([time_sig, freq_sig, mjd, dtint, lofreq, df], dtype="<f8").tobytes(),
             np.array([nchan, len(per), ptsperint], dtype="<i4").tobytes()]
    for lst in (zap_chans, zap_ints):
        a = np.asarray(sorted(lst), dtype="<i4")
        parts += [np.array([a.size], dtype="<i4").tobytes(), a.tobytes()]
    parts.append(np.array([z.size for z in per], dtype="<i4").tobytes())
    for z in per:
        if 0 < z.size < nchan:
            parts.append(z.astype("<i4").tobytes())
    with open(filename, "wb") as f:
        f.write(b"".join(parts))


def get_mask(rfimask, startsamp, N):
    """[nchan, N] bool, True = masked: every sample of interval
    floor(s / ptsperint) masks that interval's zapped channels
    (bin/waterfaller.py:28-48)."""
    blocknums = (np.arange(startsamp, startsamp + N) // rfimask.ptsperint).astype(int)
    mask = np.zeros((N, rfimask.nchan), dtype=bool)
    for b in np.unique(blocknums):
        if b < 0 or b >= len(rfimask.mask_zap_chans_per_int):
            raise IndexError("sample block %d outside the mask's %d intervals"
                             % (b, len(rfimask.mask_zap_chans_per_int)))
        sel = blocknums == b
        rows = np.zeros((int(sel.sum()), rfimask.nchan), dtype=bool)
        rows[:, np.asarray(rfimask.mask_zap_chans_per_int[b], dtype=np.intp)] = True
        mask[sel] = rows
    return mask.T
