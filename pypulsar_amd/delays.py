"""Host-side delay arithmetic, float64, bit-exact with the reference.

The reference computes every integer channel delay on the host in float64
(formats/spectra.py:126-130, 247-250) with PRESTO's ``delay_from_DM``.  These
tables are built here, in the same operation order, and uploaded as int32:
they are tiny (D x C) and must be bit-exact, so they never touch a GPU FMA.

* ``delay_from_DM(dm, f) = dm / ((0.000241 * f) * f)``  (PRESTO psr_utils; called
  at spectra.py:126-127, 247-248, waterfaller.py:160,194)
* ``dm_smear(dm, bw, f) = dm * bw / (((0.0001205 * f) * f) * f)``  (PRESTO
  psr_utils; called at DDplan2b.py:129,137,146,171,259,299,301)
* bins = ``round_half_even((delay(dm-cur, f_c) - delay(dm-cur, f_ref)) / dt)``
"""
import numpy as np

# PRESTO's dispersion constant as the reference uses it (1/k_DM in MHz^-2 s^-1 ...)
_K = 0.000241
_K_SMEAR = 0.0001205


def delay_from_DM(dm, freqs):
    """Dispersion delay in seconds (PRESTO psr_utils.delay_from_DM).

    ``freqs`` may be a scalar or an array; non-positive frequencies give 0."""
    f = np.asarray(freqs, dtype=np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        d = np.where(f > 0.0, dm / (_K * f * f), 0.0)
    return d


def dm_smear(dm, bw, fctr):
    """Smearing in seconds of ``dm`` across ``bw`` MHz at ``fctr`` MHz."""
    return dm * bw / (_K_SMEAR * fctr * fctr * fctr)


def guess_DMstep(dt, bw, fctr):
    """DM step whose smearing across ``bw`` equals ``dt`` (DDplan2b.py:438-447)."""
    return dt * 0.0001205 * fctr ** 3.0 / bw


def dedisperse_bins(dm, freqs, dt, cur_dm=0.0):
    """Integer shifts of ``Spectra.dedisperse(dm)`` (spectra.py:247-250):
    reference frequency = the highest channel frequency."""
    freqs = np.asarray(freqs, dtype=np.float64)
    ref = delay_from_DM(dm - cur_dm, np.max(freqs))
    rel = delay_from_DM(dm - cur_dm, freqs) - ref
    return np.round(rel / dt).astype(np.int64)


def subband_layout(freqs, nsub):
    """(hi, lo, ctr) frequencies of ``nsub`` contiguous subbands
    (spectra.py:119-122; channels per subband = C // nsub, the py2 '/')."""
    freqs = np.asarray(freqs, dtype=np.float64)
    cps = len(freqs) // nsub
    hi = freqs[np.arange(nsub) * cps]
    lo = freqs[(1 + np.arange(nsub)) * cps - 1]
    return hi, lo, 0.5 * (hi + lo)


def subband_bins(subdm, freqs, dt, nsub, cur_dm=0.0):
    """Integer shifts of ``Spectra.subband(nsub, subdm)`` (spectra.py:124-130):
    each channel relative to its subband's FIRST channel frequency."""
    freqs = np.asarray(freqs, dtype=np.float64)
    cps = len(freqs) // nsub
    hi, _, _ = subband_layout(freqs, nsub)
    ref = delay_from_DM(subdm - cur_dm, hi)
    rel = delay_from_DM(subdm - cur_dm, freqs) - ref.repeat(cps)
    return np.round(rel / dt).astype(np.int64)


def sweep_table(dms, freqs, dt, cur_dm=0.0):
    """[D, C] int64 table, row d = dedisperse_bins(dms[d]).

    Built with the per-element op order of ``dedisperse_bins`` (broadcast
    float64 division is correctly rounded, so rows are bit-identical)."""
    dms = np.asarray(dms, dtype=np.float64)
    freqs = np.asarray(freqs, dtype=np.float64)
    ddm = (dms - cur_dm)[:, None]
    fmax = np.max(freqs)
    with np.errstate(divide="ignore", invalid="ignore"):
        ref = np.where(fmax > 0.0, ddm / (_K * fmax * fmax), 0.0)
        d = np.where(freqs[None, :] > 0.0, ddm / (_K * freqs[None, :] * freqs[None, :]), 0.0)
    return np.round((d - ref) / dt).astype(np.int64)


def to_int32(bins):
    b = np.asarray(bins)
    if b.size and (b.max() >= 2 ** 31 or b.min() < -2 ** 31):
        raise OverflowError("delay bins do not fit int32")
    return np.ascontiguousarray(b, dtype=np.int32)
