"""ORACLE (test infrastructure only; see oracle/__init__.py).

NumPy float64 restatement of the single-pulse boxcar search of
pypulsar_amd/search.py (pdd_search.hip).  The reference holds no search: its
boxcar is Pulse.smooth (formats/pulse.py:217-241, kernel ones(w)/sqrt(w),
from PRESTO's single_pulse_search.py), followed here without wrap-around:
only starts whose whole boxcar lies inside the row are searched.  PRESTO is
absent, so parity with PRESTO's detrending and candidate pruning is
unpinned; the GPU is checked against this definition.
"""
import numpy as np

WINDOW = 1024


def chunk_stats(x, L):
    """Per row, per chunk of L samples (last may be short): mean and 1/std
    (0 where std == 0), population variance."""
    x = np.asarray(x, dtype=np.float64)
    D, n = x.shape
    nch = -(-n // L)
    mean = np.zeros((D, nch))
    istd = np.zeros((D, nch))
    for k in range(nch):
        seg = x[:, k * L:min(n, (k + 1) * L)]
        m = seg.mean(axis=1)
        v = ((seg - m[:, None]) ** 2).mean(axis=1)
        mean[:, k] = m
        istd[:, k] = np.where(v > 0, 1.0 / np.sqrt(np.where(v > 0, v, 1.0)), 0.0)
    return mean, istd


def normalise(x, L):
    """z = (x - mean_k) / std_k per chunk (pulse.py:217-241 assumes unit-RMS
    input: 'The height of the tophat is chosen such that RMS = 1')."""
    x = np.asarray(x, dtype=np.float64)
    mean, istd = chunk_stats(x, L)
    k = np.arange(x.shape[1]) // L
    return (x - mean[:, k]) * istd[:, k]


def boxcar_snr(z, w):
    """snr_w[t] = sum(z[t:t+w]) / sqrt(w) for t = 0 .. n-w  (pulse.py:232-233)."""
    c = np.concatenate([np.zeros((z.shape[0], 1)), np.cumsum(z, axis=1)], axis=1)
    return (c[:, w:] - c[:, :-w]) / np.sqrt(w)


def search(x, widths, threshold, L, window=WINDOW):
    """Candidates [(row, start, width, snr)] sorted by (row, start), plus the
    per-window margin between the best and the runner-up (width, start) --
    tests skip exact (start, width) comparison for near-ties."""
    z = normalise(x, L)
    D, n = z.shape
    nwin = -(-n // window)
    best = np.full((D, nwin), -np.inf)
    second = np.full((D, nwin), -np.inf)
    bt = np.zeros((D, nwin), dtype=np.int64)
    bw = np.zeros((D, nwin), dtype=np.int64)
    for w in widths:
        if w > n:
            break
        s = boxcar_snr(z, w)  # [D, n-w+1]
        m = s.shape[1]
        pad = nwin * window - m
        sp = np.concatenate([s, np.full((D, pad), -np.inf)], axis=1).reshape(D, nwin, window)
        top2 = np.sort(sp, axis=2)[:, :, -2:]
        arg = sp.argmax(axis=2)  # first (smallest start) among ties
        val = top2[:, :, 1]
        # runner-up over everything seen so far
        second = np.maximum(second, np.where(val > best, best, val))
        second = np.maximum(second, top2[:, :, 0])
        upd = val > best  # strict: ties keep the smaller width
        best = np.where(upd, val, best)
        bt = np.where(upd, np.arange(nwin)[None, :] * window + arg, bt)
        bw = np.where(upd, w, bw)
    out, margin = [], []
    for d in range(D):
        for k in range(nwin):
            if np.isfinite(best[d, k]) and best[d, k] >= threshold:
                out.append((d, int(bt[d, k]), int(bw[d, k]), float(best[d, k])))
                margin.append(float(best[d, k] - second[d, k]))
    return out, margin
