#!/usr/bin/env python
"""Generate tests/golden/golden_psrfits.npz: the reference's OWN PSRFITS decode
(/root/reference/formats/psrfits.py:37-50 unpack_4bit, :89-107 read_subint,
:143-183 get_spectra) on small synthetic subints, so the device decode
(k_psrfits_subints) and oracle/psrfits_oracle.py are pinned to the reference
and not only to each other.

RUN ONLY IN THE BUILD CONTAINER (it executes the read-only reference, which
never travels to the GPU box).  Only the .npz this script writes is committed.

How the reference runs here: psrfits.py imports pyslalib, psr_utils,
pypulsar.utils.astro.protractor, pypulsar.formats.spectra, astropy.io.fits
and memory.  Probe-only stand-ins are put in sys.modules for the ones that are
absent (none of them is called by the functions exercised): empty
pyslalib/protractor/astropy.io.fits/memory modules, the psr_utils restatement
of make_golden.py, and for pypulsar.formats.spectra the reference's own
spectra.py loaded as make_golden.py loads it.  PsrfitsFile.__init__ opens the
file with astropy (absent), so instances are made with __new__ and given the
attributes __init__ would set; ``fits`` is a stand-in whose
fits['SUBINT'].data[isub][column] returns the column values astropy returns
for a search-mode SUBINT row: DATA as stored (uint8 bytes, 4-bit packed low
nibble first; big-endian int16 for 16 bits; big-endian float32 for 32 bits),
DAT_SCL / DAT_OFFS / DAT_WTS as big-endian float32, DAT_FREQ float64.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_psrfits.py
"""
import importlib.util
import os
import sys
import types

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

import make_golden  # noqa: E402

NSUB, NSBLK, NCHAN, DT = 4, 40, 24, 64e-6
SPANS = [(0, NSBLK), (7, 2 * NSBLK), (NSBLK, NSBLK // 2), (0, 3 * NSBLK), (NSBLK - 1, 2),
         (5, 0), (3, NSBLK - 3)]


def load_psrfits():
    spectra, _, _ = make_golden.load_reference()   # also puts the psr_utils probe on sys.path
    for name in ("pyslalib", "pyslalib.slalib", "memory", "astropy", "astropy.io",
                 "astropy.io.fits", "pypulsar", "pypulsar.utils", "pypulsar.utils.astro",
                 "pypulsar.utils.astro.protractor", "pypulsar.formats"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["pyslalib"].slalib = sys.modules["pyslalib.slalib"]
    sys.modules["astropy"].io = sys.modules["astropy.io"]
    sys.modules["astropy.io"].fits = sys.modules["astropy.io.fits"]
    sys.modules["pypulsar.utils.astro"].protractor = sys.modules["pypulsar.utils.astro.protractor"]
    sys.modules["pypulsar.formats.spectra"] = spectra
    sys.modules["pypulsar.formats"].spectra = spectra
    spec = importlib.util.spec_from_file_location(
        "ref_psrfits", os.path.join(make_golden.REF, "formats", "psrfits.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


class _Subint(object):
    def __init__(self, rows):
        self.data = rows


class _Fits(object):
    def __init__(self, rows):
        self._sub = _Subint(rows)

    def __getitem__(self, key):
        assert key == "SUBINT"
        return self._sub


def stored(data, nbits):
    """[nsub, nsblk, nchan] samples -> the DATA column values as stored."""
    flat = data.reshape(data.shape[0], -1)
    if nbits == 4:
        return ((flat[:, 0::2] & 15) | ((flat[:, 1::2] & 15) << 4)).astype(np.uint8)
    return flat.astype({8: np.uint8, 16: ">i2", 32: ">f4"}[nbits])


def case_inputs(nbits, ascending, seed):
    rng = np.random.default_rng(seed)
    if nbits == 16:
        data = rng.integers(-3000, 3000, (NSUB, NSBLK, NCHAN)).astype(np.int16)
    elif nbits == 32:
        data = rng.normal(0, 5, (NSUB, NSBLK, NCHAN)).astype(np.float32)
    else:
        data = rng.integers(0, {4: 16, 8: 256}[nbits], (NSUB, NSBLK, NCHAN)).astype(np.uint8)
    f = 1200.0 + 2.0 * np.arange(NCHAN)
    freqs = f if ascending else f[::-1].copy()
    scl = rng.uniform(0.5, 2.0, (NSUB, NCHAN)).astype(np.float32)
    off = rng.uniform(-3, 3, (NSUB, NCHAN)).astype(np.float32)
    wts = rng.choice([0.0, 1.0, 0.5], (NSUB, NCHAN)).astype(np.float32)
    return data, freqs, scl, off, wts


def ref_file(ref, data, nbits, freqs, scl, off, wts):
    body = stored(data, nbits)
    rows = [{"DATA": body[i], "DAT_SCL": scl[i].astype(">f4"), "DAT_OFFS": off[i].astype(">f4"),
             "DAT_WTS": wts[i].astype(">f4"), "DAT_FREQ": freqs.astype(np.float64)}
            for i in range(NSUB)]
    pf = ref.PsrfitsFile.__new__(ref.PsrfitsFile)
    pf.fits = _Fits(rows)
    pf.nbits = nbits
    pf.nchan = NCHAN
    pf.nsamp_per_subint = NSBLK
    pf.nsubints = NSUB
    pf.freqs = rows[0]["DAT_FREQ"]
    pf.frequencies = pf.freqs
    pf.tsamp = DT
    # SpectraInfo (psrfits.py:459-464): the band is flipped when the header's
    # high frequency is below its low one, i.e. DAT_FREQ descends
    pf.specinfo = types.SimpleNamespace(need_flipband=bool(freqs[0] > freqs[-1]))
    return pf


def main():
    ref = load_psrfits()
    fx = {}
    # unpack_4bit on every byte value
    b = np.arange(256, dtype=np.uint8)
    fx["unpack4_in"] = b
    fx["unpack4_out"] = np.asarray(ref.unpack_4bit(b))
    for nbits in (4, 8, 16, 32):
        for asc in (True, False):
            key = "b%d_%s" % (nbits, "asc" if asc else "desc")
            data, freqs, scl, off, wts = case_inputs(nbits, asc, 100 + nbits + asc)
            fx[key + "_data"] = data
            fx[key + "_freqs"] = freqs
            fx[key + "_scl"], fx[key + "_off"], fx[key + "_wts"] = scl, off, wts
            pf = ref_file(ref, data, nbits, freqs, scl, off, wts)
            fx[key + "_flip"] = np.array(pf.specinfo.need_flipband)
            for isub in (0, 3):
                out = pf.read_subint(isub)
                assert out.dtype == np.float32
                fx["%s_sub%d" % (key, isub)] = out
            for k, (start, n) in enumerate(SPANS):
                s = pf.get_spectra(start, n)
                fx["%s_span%d" % (key, k)] = np.asarray(s.data)          # float64 [nchan, n]
                fx["%s_span%d_freqs" % (key, k)] = np.asarray(s.freqs)
                fx["%s_span%d_start" % (key, k)] = np.array(s.starttime)
            if nbits == 8:
                fx[key + "_flags"] = pf.read_subint(1, apply_weights=False, apply_scales=True,
                                                    apply_offsets=False)
    fx["spans"] = np.array(SPANS)
    fx["geom"] = np.array([NSUB, NSBLK, NCHAN])
    np.savez_compressed(os.path.join(HERE, "golden_psrfits.npz"), **fx)
    print("wrote %d arrays" % len(fx))


if __name__ == "__main__":
    main()
