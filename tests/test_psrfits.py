"""CPU tests of the PSRFITS host side: the FITS container codec
(formats/fits.py), SpectraInfo / header parsing (formats/psrfits.py:186-464),
the calendar and sexagesimal conversions, unpack_4bit against the oracle.
No PSRFITS file ships with the reference: files are written by
write_search_psrfits and read back (parity with real files unpinned)."""
import numpy as np
import pytest

from oracle import psrfits_oracle as po


def _mkfile(tmp_path, nbits=8, nsub=3, nsblk=64, nchan=16, ascending=True, seed=0):
    from pypulsar_amd.formats.psrfits import write_search_psrfits
    rng = np.random.default_rng(seed)
    hi = {4: 16, 8: 256}.get(nbits)
    if nbits == 16:
        data = rng.integers(-3000, 3000, (nsub, nsblk, nchan)).astype(np.int16)
    elif nbits == 32:
        data = rng.normal(0, 5, (nsub, nsblk, nchan)).astype(np.float32)
    else:
        data = rng.integers(0, hi, (nsub, nsblk, nchan)).astype(np.uint8)
    f = 1200.0 + 2.0 * np.arange(nchan)
    freqs = f if ascending else f[::-1]
    scl = rng.uniform(0.5, 2.0, (nsub, nchan)).astype(np.float32)
    off = rng.uniform(-3, 3, (nsub, nchan)).astype(np.float32)
    wts = rng.choice([0.0, 1.0, 0.5], (nsub, nchan)).astype(np.float32)
    fn = str(tmp_path / ("t%d.fits" % nbits))
    write_search_psrfits(fn, data, freqs, 64e-6, nbits, scl, off, wts)
    return fn, data, freqs, scl, off, wts


def test_fits_roundtrip(tmp_path):
    from pypulsar_amd.formats import fits
    fn, data, freqs, scl, off, wts = _mkfile(tmp_path, nbits=16)
    h = fits.open(fn)
    assert [x.name for x in h] == ["PRIMARY", "SUBINT"]
    assert h["PRIMARY"].header["FITSTYPE"] == "PSRFITS"
    assert h["PRIMARY"].header["DATE-OBS"] == "2020-01-02T03:04:05.500"
    assert h["PRIMARY"].header["STT_OFFS"] == 0.5
    sub = h["SUBINT"]
    assert sub.columns.names[-1] == "DATA" and sub.columns[-1].format.endswith("I")
    np.testing.assert_array_equal(sub.data[1]["DAT_FREQ"], freqs)
    np.testing.assert_array_equal(sub.data[2]["DAT_SCL"], scl[2])
    np.testing.assert_array_equal(sub.data[0]["DATA"], data[0].reshape(-1))
    assert sub.raw_rows(0, 3).shape == (3, sub.header["NAXIS1"])


def test_card_values():
    from pypulsar_amd.formats import fits
    assert fits._parse_value("'it''s   '  / c") == "it's"
    assert fits._parse_value("                   T") is True
    assert fits._parse_value("  42 / answer") == 42
    assert fits._parse_value("  1.5D3") == 1500.0


def test_spectrainfo(tmp_path):
    from pypulsar_amd.formats.psrfits import SpectraInfo, is_PSRFITS
    fn, data, freqs, scl, off, wts = _mkfile(tmp_path, nbits=4, nsub=5, nsblk=32, nchan=8)
    assert is_PSRFITS(fn)
    si = SpectraInfo([fn])
    assert si.num_channels == 8 and si.spectra_per_subint == 32 and si.bits_per_sample == 4
    assert si.N == 5 * 32 and si.T == pytest.approx(160 * 64e-6)
    assert si.need_scale and si.need_offset and si.need_weight
    assert not si.need_flipband and si.lo_freq < si.hi_freq
    assert si.start_MJD[0] == pytest.approx(58850 + 11045.5 / 86400.0)
    assert si.ra2000 == pytest.approx((12 + 34 / 60 + 56.7 / 3600) * 15)
    assert si.dec2000 == pytest.approx(-(1 + 23 / 60 + 45.6 / 3600))
    assert si.summed_polns and si.FITS_typecode == "B"
    txt = str(si)
    assert "Number of channels = 8" in txt and "Need band inverted? = False" in txt
    fn2 = _mkfile(tmp_path, nbits=8, ascending=False)[0]
    assert SpectraInfo([fn2]).need_flipband


def test_calendar():
    from pypulsar_amd.formats.psrfits import DATEOBS_to_MJD, _cldj
    assert _cldj(2000, 1, 1) == (51544.0, 0)
    assert _cldj(1858, 11, 17) == (0.0, 0)
    assert _cldj(2020, 2, 30)[1] == 3
    day, frac = DATEOBS_to_MJD("2020-01-02T06:00:00")
    assert day == 58850.0 and frac == pytest.approx(0.25)


def test_unpack_4bit():
    from pypulsar_amd.formats.psrfits import unpack_4bit
    b = np.array([0x21, 0xF0, 0x0E], dtype=np.uint8)
    np.testing.assert_array_equal(unpack_4bit(b), [1, 2, 0, 15, 14, 0])
    np.testing.assert_array_equal(unpack_4bit(b), po.unpack_4bit(b))


def test_not_psrfits(tmp_path):
    from pypulsar_amd.formats import fits
    from pypulsar_amd.formats.psrfits import SpectraInfo, is_PSRFITS
    fn = str(tmp_path / "x.fits")
    fits.write(fn, [("OBS_MODE", "PSR")], [])
    assert not is_PSRFITS(fn)
    with pytest.raises(ValueError):
        SpectraInfo([fn])


GOLD = None


def _gold():
    global GOLD
    if GOLD is None:
        import os
        GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_psrfits.npz"))
    return GOLD


def _stored(data, nbits):
    flat = data.reshape(data.shape[0], -1)
    if nbits == 4:
        return ((flat[:, 0::2] & 15) | ((flat[:, 1::2] & 15) << 4)).astype(np.uint8)
    return flat.astype({8: np.uint8, 16: ">i2", 32: ">f4"}[nbits])


@pytest.mark.parametrize("nbits", [4, 8, 16, 32])
@pytest.mark.parametrize("order", ["asc", "desc"])
def test_oracle_matches_reference_fixtures(nbits, order):
    """oracle/psrfits_oracle.py against the reference's own read_subint /
    get_spectra outputs (tests/golden/make_golden_psrfits.py executed
    /root/reference/formats/psrfits.py:37-183): bit-exact."""
    g = _gold()
    key = "b%d_%s" % (nbits, order)
    nsub, nsblk, nchan = (int(v) for v in g["geom"])
    data, freqs = g[key + "_data"], g[key + "_freqs"]
    scl, off, wts = g[key + "_scl"], g[key + "_off"], g[key + "_wts"]
    body = _stored(data, nbits)
    subs = [po.read_subint(body[i], nbits, nsblk, nchan, scl[i].astype(">f4"),
                           off[i].astype(">f4"), wts[i].astype(">f4")) for i in range(nsub)]
    for isub in (0, 3):
        np.testing.assert_array_equal(subs[isub], g["%s_sub%d" % (key, isub)])
        assert subs[isub].dtype == g["%s_sub%d" % (key, isub)].dtype == np.float32
    for k, (start, n) in enumerate(g["spans"]):
        want = g["%s_span%d" % (key, k)]
        got, gf = po.get_spectra(subs, nsblk, freqs, bool(g[key + "_flip"]), int(start), int(n))
        np.testing.assert_array_equal(np.asarray(got, dtype=np.float64), want)
        np.testing.assert_array_equal(gf, g["%s_span%d_freqs" % (key, k)])
    if nbits == 8:
        got = po.read_subint(body[1], 8, nsblk, nchan, scl[1], off[1], wts[1], apply_weights=False,
                             apply_offsets=False)
        np.testing.assert_array_equal(got, g[key + "_flags"])


def test_unpack_4bit_reference_fixture():
    from pypulsar_amd.formats.psrfits import unpack_4bit
    g = _gold()
    np.testing.assert_array_equal(unpack_4bit(g["unpack4_in"]), g["unpack4_out"])
    np.testing.assert_array_equal(po.unpack_4bit(g["unpack4_in"]), g["unpack4_out"])


@pytest.mark.parametrize("order", ["asc", "desc"])
def test_spectrainfo_flipband_matches_reference_case(tmp_path, order):
    """The header this repo's writer produces for the fixture band gives the
    need_flipband the reference case used (psrfits.py:459-464)."""
    from pypulsar_amd.formats.psrfits import SpectraInfo, write_search_psrfits
    g = _gold()
    key = "b8_%s" % order
    fn = str(tmp_path / "f.fits")
    write_search_psrfits(fn, g[key + "_data"], g[key + "_freqs"], 64e-6, 8, g[key + "_scl"],
                         g[key + "_off"], g[key + "_wts"])
    assert SpectraInfo([fn]).need_flipband == bool(g[key + "_flip"])
