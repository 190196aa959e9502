"""PSRFITS on the GPU: PsrfitsFile.read_subint / get_spectra through
pdd_psrfits_subints against the oracle restatement of psrfits.py:67-183,
bit-exact (the same float32 operations in the same order), for 4/8/16/32-bit
data, both band orders and spans across subint boundaries; then the device
Spectra runs the dedispersion hot path."""
import numpy as np
import pytest

from oracle import psrfits_oracle as po
from test_psrfits import _mkfile

pytestmark = pytest.mark.gpu


def _oracle_subints(data, nbits, scl, off, wts):
    out = []
    for i in range(data.shape[0]):
        raw = data[i].reshape(-1)
        if nbits == 4:  # as stored: two samples per byte, low nibble first
            raw = (raw[0::2] & 15) | ((raw[1::2] & 15) << 4)
        out.append(po.read_subint(raw.astype({4: np.uint8, 8: np.uint8, 16: ">i2",
                                              32: ">f4"}[nbits]),
                                  nbits, data.shape[1], data.shape[2], scl[i], off[i], wts[i]))
    return out


@pytest.mark.parametrize("nbits", [4, 8, 16, 32])
@pytest.mark.parametrize("ascending", [True, False])
def test_get_spectra(gpu, tmp_path, nbits, ascending):
    from pypulsar_amd.formats.psrfits import PsrfitsFile
    fn, data, freqs, scl, off, wts = _mkfile(tmp_path, nbits=nbits, nsub=4, nsblk=100, nchan=70,
                                             ascending=ascending, seed=nbits)
    pf = PsrfitsFile(fn)
    subs = _oracle_subints(data, nbits, scl, off, wts)
    for i in (0, 3):
        np.testing.assert_array_equal(pf.read_subint(i), subs[i].astype(np.float32))
    for start, N in [(0, 100), (37, 150), (150, 50), (0, 400), (99, 2), (250, 149), (10, 0)]:
        s = pf.get_spectra(start, N)
        want, wf = po.get_spectra(subs, 100, np.array(freqs), pf.specinfo.need_flipband, start, N)
        assert s.data.shape == (70, N)
        np.testing.assert_array_equal(s.device_data.cpu().numpy(), want.astype(np.float32))
        np.testing.assert_array_equal(s.freqs, wf)
        assert s.starttime == pytest.approx(start * 64e-6) and s.dt == 64e-6
        assert s.freqs[0] > s.freqs[-1] or N == 0


def test_read_subint_flags(gpu, tmp_path):
    from pypulsar_amd.formats.psrfits import PsrfitsFile
    fn, data, freqs, scl, off, wts = _mkfile(tmp_path, nbits=8, nsub=2, nsblk=64, nchan=16)
    pf = PsrfitsFile(fn)
    got = pf.read_subint(1, apply_weights=False, apply_scales=True, apply_offsets=False)
    raw = data[1].reshape(-1)
    want = po.read_subint(raw, 8, 64, 16, scl[1], off[1], wts[1], apply_weights=False,
                          apply_offsets=False)
    np.testing.assert_array_equal(got, want.astype(np.float32))


def test_psrfits_then_dedisperse(gpu, tmp_path):
    """The device Spectra from a PSRFITS file feeds the hot path unchanged."""
    from oracle import spectra_oracle as orc
    from pypulsar_amd.formats.psrfits import PsrfitsFile
    fn, data, freqs, scl, off, wts = _mkfile(tmp_path, nbits=8, nsub=4, nsblk=256, nchan=32)
    pf = PsrfitsFile(fn)
    s = pf.get_spectra(10, 900)
    x = s.device_data.cpu().numpy().astype(np.float64)
    s.dedisperse(20.0, padval=0, trim=True)
    want, _ = orc.dedisperse(x, np.asarray(s.freqs), s.dt, 20.0, padval=0, trim=True)
    got = s.data
    assert got.shape == want.shape
    assert np.max(np.abs(got - want)) <= 1e-5 * np.max(np.abs(want))


@pytest.mark.parametrize("nbits", [4, 8, 16, 32])
@pytest.mark.parametrize("order", ["asc", "desc"])
def test_device_decode_matches_reference_fixtures(gpu, tmp_path, nbits, order):
    """k_psrfits_subints (through PsrfitsFile.read_subint / get_spectra of a
    file holding the fixture's subints) against the REFERENCE's own outputs
    (tests/golden/golden_psrfits.npz, made by executing
    /root/reference/formats/psrfits.py:37-183): bit-exact float32 values,
    frequencies and start times (f3 pinned)."""
    import os
    from pypulsar_amd.formats.psrfits import PsrfitsFile, write_search_psrfits
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_psrfits.npz"))
    key = "b%d_%s" % (nbits, order)
    fn = str(tmp_path / ("%s.fits" % key))
    write_search_psrfits(fn, g[key + "_data"], g[key + "_freqs"], 64e-6, nbits, g[key + "_scl"],
                         g[key + "_off"], g[key + "_wts"])
    pf = PsrfitsFile(fn)
    assert pf.specinfo.need_flipband == bool(g[key + "_flip"])
    for isub in (0, 3):
        np.testing.assert_array_equal(pf.read_subint(isub), g["%s_sub%d" % (key, isub)])
    for k, (start, n) in enumerate(g["spans"]):
        s = pf.get_spectra(int(start), int(n))
        np.testing.assert_array_equal(s.device_data.cpu().numpy().astype(np.float64),
                                      g["%s_span%d" % (key, k)])
        np.testing.assert_array_equal(s.freqs, g["%s_span%d_freqs" % (key, k)])
        assert s.starttime == float(g["%s_span%d_start" % (key, k)])
    if nbits == 8:
        got = pf.read_subint(1, apply_weights=False, apply_scales=True, apply_offsets=False)
        np.testing.assert_array_equal(got, g[key + "_flags"])
