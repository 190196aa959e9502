"""ORACLE (test infrastructure only; see oracle/__init__.py).

NumPy restatement of the reference's Spectra hot path, float64 like the
reference.  Each function cites the reference lines it follows.  Functions take
and return plain arrays (no class state) so tests can compose them exactly the
way the reference methods compose.
"""
import numpy as np

# --------------------------------------------------------------------------
# PRESTO psr_utils (not in the reference tree; restated; parity unpinned)
# call sites: formats/spectra.py:80,126-127,247-248; utils/DDplan2b.py:129..382
# --------------------------------------------------------------------------


def delay_from_DM(dm, freqs):
    """PRESTO psr_utils.delay_from_DM: DM / (0.000241 * f * f), 0 where f<=0.

    Evaluated left to right, (0.000241*f)*f, in float64."""
    f = np.asarray(freqs, dtype=np.float64)
    with np.errstate(divide="ignore"):
        return np.where(f > 0.0, dm / (0.000241 * f * f), 0.0)


def rotate(arr, bins):
    """PRESTO psr_utils.rotate: left rotation by ``bins mod len``."""
    n = len(arr)
    b = int(bins) % n
    if b == 0:
        return arr
    return np.concatenate((arr[b:], arr[:b]))


def dm_smear(dm, bw, fctr):
    """PRESTO psr_utils.dm_smear: DM*BW/(0.0001205*f*f*f) seconds."""
    return dm * bw / (0.0001205 * fctr * fctr * fctr)


# --------------------------------------------------------------------------
# formats/spectra.py
# --------------------------------------------------------------------------


def dedisperse_bins(dm, cur_dm, freqs, dt):
    """Delay-bin table of Spectra.dedisperse, spectra.py:247-250."""
    freqs = np.asarray(freqs, dtype=np.float64)
    ref = delay_from_DM(dm - cur_dm, np.max(freqs))
    rel = delay_from_DM(dm - cur_dm, freqs) - ref
    return np.round(rel / dt).astype(np.int64)


def subband_bins(subdm, cur_dm, freqs, dt, nsub):
    """Delay-bin table of Spectra.subband, spectra.py:119-130 (py2 '/')."""
    freqs = np.asarray(freqs, dtype=np.float64)
    cps = len(freqs) // nsub
    hi = freqs[np.arange(nsub) * cps]
    ref = delay_from_DM(subdm - cur_dm, hi)
    rel = delay_from_DM(subdm - cur_dm, freqs) - ref.repeat(cps)
    return np.round(rel / dt).astype(np.int64)


def subband_freqs(freqs, nsub):
    """Subband centre frequencies, spectra.py:119-122,137."""
    cps = len(freqs) // nsub
    hi = freqs[np.arange(nsub) * cps]
    lo = freqs[(1 + np.arange(nsub)) * cps - 1]
    return 0.5 * (hi + lo)


def shift_channels(data, bins, padval=0):
    """Spectra.shift_channels, spectra.py:54-94 (per-channel loop, in place
    on a copy).  Pad value for 'mean'/'median' is computed on the rotated
    channel, before padding (spectra.py:80-86)."""
    out = np.array(data, dtype=np.float64, copy=True)
    assert out.shape[0] == len(bins)
    for ii in range(out.shape[0]):
        chan = out[ii]
        b = int(bins[ii])
        chan[:] = rotate(chan, b)
        if isinstance(padval, str) and padval == "rotate":
            continue
        if isinstance(padval, str) and padval == "mean":
            pad = np.mean(chan)
        elif isinstance(padval, str) and padval == "median":
            pad = np.median(chan)
        else:
            pad = padval
        if b > 0:
            chan[-b:] = pad
        elif b < 0:
            chan[:-b] = pad
    return out


def dedisperse(data, freqs, dt, dm, cur_dm=0.0, padval=0, trim=False):
    """Spectra.dedisperse, spectra.py:229-260.  Returns (data, new_dm)."""
    assert dm >= 0
    bins = dedisperse_bins(dm, cur_dm, freqs, dt)
    out = shift_channels(data, bins, padval)
    if trim:
        ntrim = max(bins)
        if ntrim > 0:
            out = out[:, :-ntrim]
    return out, dm


def subband(data, freqs, dt, nsub, subdm=None, cur_dm=0.0, padval=0):
    """Spectra.subband, spectra.py:96-138.  Returns (data, new_freqs);
    the Spectra's dm is NOT changed by subband."""
    C = data.shape[0]
    assert C % nsub == 0
    assert subdm is None or subdm >= 0
    out = np.asarray(data, dtype=np.float64)
    if subdm is not None:
        out = shift_channels(out, subband_bins(subdm, cur_dm, freqs, dt, nsub), padval)
    out = np.array([np.sum(s, axis=0) for s in np.vsplit(out, nsub)])
    return out, subband_freqs(np.asarray(freqs, dtype=np.float64), nsub)


def trim(data, nbins, starttime, dt):
    """Spectra.trim, spectra.py:305-327.  Returns (data, numspectra,
    starttime); keeps the reference's bins<0 numspectra arithmetic."""
    n = data.shape[1]
    assert nbins < n
    if nbins == 0:
        return data, n, starttime
    if nbins > 0:
        return data[:, :-nbins], n - nbins, starttime
    return data[:, nbins:], n - nbins, starttime + nbins * dt


def downsample(data, dt, factor=1, trim_=True):
    """Spectra.downsample, spectra.py:329-351 (py2 '/').  Returns (data, dt)."""
    n = data.shape[1]
    assert trim_ or not (n % factor)
    new_n = n // factor
    rem = n % factor
    if rem:
        data = data[:, :-rem]
    out = data.reshape(data.shape[0], new_n, factor).sum(axis=2)
    return out, dt * factor


def channel_sum(data):
    """Dedispersed series, bin/waterfaller.py:140 (data.data.sum(axis=0))."""
    return np.asarray(data, dtype=np.float64).sum(axis=0)


# --------------------------------------------------------------------------
# bin/zero_dm_filter.py:30-39
# --------------------------------------------------------------------------


def zero_dm_filter(spectrum):
    """One spectrum (all channels at one time sample): subtract the mean,
    rounded half-even and cast to the data dtype when that differs (integer
    data wraps modulo 2**nbits)."""
    avg = spectrum.mean()
    if avg.dtype != spectrum.dtype:
        avg = np.round(avg).astype(spectrum.dtype)
    return spectrum - avg


def zero_dm_block(block):
    """zero_dm_filter applied to every spectrum of a [nspec, nchan] block
    (bin/zero_dm_filter.py:42-50 loop)."""
    return np.array([zero_dm_filter(row) for row in block])


# --------------------------------------------------------------------------
# batched sweep (new; spec = per-DM dedisperse(trim) + channel sum)
# --------------------------------------------------------------------------


def sweep_table(dms, freqs, dt, cur_dm=0.0):
    """[D, C] int64 table: row d = dedisperse_bins(dms[d])."""
    return np.array([dedisperse_bins(dm, cur_dm, freqs, dt) for dm in dms], dtype=np.int64)


def shifted_sum(data, bins, padval=0):
    """Vectorised a4+a6: sum_c shift_channels(data, bins, padval)[c] (fast
    restatement used for larger test sizes; equals channel_sum(shift_channels))."""
    data = np.asarray(data, dtype=np.float64)
    C, N = data.shape
    t = np.arange(N)
    acc = np.zeros(N, dtype=np.float64)
    for c in range(C):
        b = int(bins[c])
        if isinstance(padval, str) and padval == "rotate":
            acc += data[c, (t + b) % N]
            continue
        if isinstance(padval, str) and padval == "mean":
            pad = np.mean(data[c])
        elif isinstance(padval, str) and padval == "median":
            pad = np.median(data[c])
        else:
            pad = float(padval)
        s = t + b
        ok = (s >= 0) & (s < N)
        row = np.full(N, pad)
        row[ok] = data[c, s[ok]]
        acc += row
    return acc


def sweep_plane(data, table, padval=0, n_out=None):
    """plane[d, t] = sum_c X(c, t + table[d, c]), t < n_out.  Default n_out =
    N - max(0, max table): every row is then the prefix of the reference's
    dedisperse(trim=True) series."""
    data = np.asarray(data, dtype=np.float64)
    N = data.shape[1]
    if n_out is None:
        n_out = N - max(0, int(np.max(table)))
    return np.array([shifted_sum(data, table[d], padval)[:n_out] for d in range(table.shape[0])])


def sweep_rows_inside(data, table, n_out):
    """sweep_plane rows for trials whose reads t + table[d, c], t < n_out, all
    fall inside [0, N) (no pad is read; the trim=True rows of a grid with
    delays >= 0): the same sums as shifted_sum, taken as channel slices with
    exact int64 accumulation for integer data -- fast enough for 4096-channel
    rows at full length."""
    data = np.asarray(data)
    C, N = data.shape
    table = np.atleast_2d(np.asarray(table))
    integer = np.issubdtype(data.dtype, np.integer)
    out = np.zeros((table.shape[0], n_out), dtype=np.int64 if integer else np.float64)
    for d in range(table.shape[0]):
        acc = out[d]
        for c in range(C):
            b = int(table[d, c])
            assert 0 <= b and b + n_out <= N, "row %d reads a pad (bin %d)" % (d, b)
            acc += data[c, b:b + n_out]
    return out.astype(np.float64)


# --------------------------------------------------------------------------
# waterfaller post-chain (formats/spectra.py:140-227, 262-303)
# --------------------------------------------------------------------------


def scaled(data, indep=False):
    """Spectra.scaled, spectra.py:140-163: per channel (chan - median) / std,
    std of the whole array (indep=False) or of the channel (indep=True)."""
    out = np.array(data, dtype=np.float64, copy=True)
    if not indep:
        std = out.std()
    for ii in range(out.shape[0]):
        chan = out[ii]
        median = np.median(chan)
        if indep:
            std = chan.std()
        chan[:] = (chan - median) / std
    return out


def scaled2(data, indep=False):
    """Spectra.scaled2, spectra.py:165-188: (chan - chan.min()) / max, max of
    the whole array (indep=False) or of the channel."""
    out = np.array(data, dtype=np.float64, copy=True)
    if not indep:
        mx = out.max()
    for ii in range(out.shape[0]):
        chan = out[ii]
        mn = chan.min()
        if indep:
            mx = chan.max()
        chan[:] = (chan - mn) / mx
    return out


def mask_values(data, maskval="median-mid80"):
    """Per-channel replacement values of Spectra.masked, spectra.py:211-224.
    'median-mid80' is the median of sorted(chan)[n:-n], n = round(0.1 N):
    symmetric trimming keeps the median, except n == 0, where the slice is
    empty and the reference gets NaN."""
    data = np.asarray(data, dtype=np.float64)
    C, N = data.shape
    vals = np.ones(C)
    for ii in range(C):
        chan = data[ii]
        if maskval == "mean":
            vals[ii] = np.mean(chan)
        elif maskval == "median":
            vals[ii] = np.median(chan)
        elif maskval == "median-mid80":
            n = int(np.round(0.1 * N))
            vals[ii] = np.median(np.sort(chan)[n:-n]) if n > 0 else np.nan
        else:
            vals[ii] = maskval
    return vals


def masked(data, mask, maskval="median-mid80"):
    """Spectra.masked, spectra.py:190-227."""
    data = np.asarray(data, dtype=np.float64)
    assert data.shape == mask.shape
    vals = mask_values(data, maskval)
    return np.where(mask, np.ones_like(data) * vals[:, np.newaxis], data)


def smooth(data, width=1, padval=0):
    """Spectra.smooth, spectra.py:262-303: per channel, pad `width` samples on
    each side ('wrap', 'mean', 'median' or a number), convolve with a boxcar of
    height 1/sqrt(width) ('same' centring), keep the middle N samples."""
    out = np.array(data, dtype=np.float64, copy=True)
    if width <= 1:
        return out
    kernel = np.ones(width) / np.sqrt(width)
    N = out.shape[1]
    for ii in range(out.shape[0]):
        chan = out[ii]
        if padval == "wrap":
            tosmooth = np.concatenate([chan[-width:], chan, chan[:width]])
        else:
            if padval == "mean":
                pv = np.mean(chan)
            elif padval == "median":
                pv = np.median(chan)
            else:
                pv = padval
            tosmooth = np.ones(N + 2 * width) * pv
            tosmooth[width:-width] = chan
        chan[:] = np.convolve(tosmooth, kernel, "same")[width:-width]
    return out


# --------------------------------------------------------------------------
# streaming pipeline (new): zero-DM in float mode
# (bin/zero_dm_filter.py:35 mean, without the integer cast) + downsample
# (formats/spectra.py:329-351) of a time-major block
# --------------------------------------------------------------------------


def zdm_downsample(block_tc, factor, zero_dm=True):
    """[nspec, nchan] time-major block -> [nchan, nspec // factor] float64."""
    x = np.asarray(block_tc, dtype=np.float64)
    if zero_dm:
        x = x - x.mean(axis=1, keepdims=True)
    n = (x.shape[0] // factor) * factor
    return x[:n].reshape(n // factor, factor, x.shape[1]).sum(axis=1).T


def zdm_int_downsample(block_tc, factor, mode="int"):
    """Integer prologue of the stream's exact 16-bit path: [nspec, nchan]
    uint8 -> [nchan, nspec // factor] int64 co-added values, zero-DM by mode:
      'wrap': zero_dm_block (bin/zero_dm_filter.py:30-39 on uint8 data,
              the reference's result exactly: wraps modulo 256);
      'int':  x - np.round(mean) as a signed integer (the reference's rounded
              mean, :35-38, without the uint8 cast of the difference);
      'none': x.
    Downsample = co-add of ``factor`` spectra (formats/spectra.py:329-351)."""
    x = np.asarray(block_tc)
    assert x.dtype == np.uint8
    if mode == "wrap":
        z = zero_dm_block(x).astype(np.int64)
    elif mode == "int":
        avg = np.array([np.round(row.mean()) for row in x])  # per spectrum, as :35-38
        z = x.astype(np.int64) - avg.astype(np.int64)[:, None]
    else:
        z = x.astype(np.int64)
    n = (z.shape[0] // factor) * factor
    return z[:n].reshape(n // factor, factor, z.shape[1]).sum(axis=1).T
