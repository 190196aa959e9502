"""Drop-in API fidelity on the GPU: the reference's data-access idioms.

formats/spectra.py:42-52 returns VIEWS into the Spectra's ndarray
(``get_chan``/``get_spectrum``/``data[...]``), so callers may write through
them; the device-resident Spectra must either see those writes or refuse
them loudly -- never drop them silently."""
import numpy as np
import pytest

from conftest import band, u8_data

DT = 64e-6
pytestmark = pytest.mark.gpu


def test_get_chan_write_through(gpu):
    from pypulsar_amd.formats.spectra import Spectra
    C, N = 16, 512
    x = u8_data(C, N, 4)
    s = Spectra(band(C), DT, x)
    chan = s.get_chan(3)
    chan[:] = 7.0                       # the reference idiom
    np.testing.assert_array_equal(s.get_chan(3), np.full(N, 7.0))
    assert float(s.device_data[3].min()) == float(s.device_data[3].max()) == 7.0
    c5 = s.get_chan(5)
    c5 += 1.0                           # in-place arithmetic
    np.testing.assert_array_equal(s.get_chan(5), x[5].astype(np.float64) + 1.0)
    spec = s.get_spectrum(10)
    spec[:4] = -1.0
    np.testing.assert_array_equal(s.data[:4, 10], -1.0)
    d = s.data
    d[1][2:4] = 9.0                     # slice of a row of the view
    d[2, 5:9] = 3.0
    got = s.data
    np.testing.assert_array_equal(got[1, 2:4], 9.0)
    np.testing.assert_array_equal(got[2, 5:9], 3.0)
    # other channels untouched
    np.testing.assert_array_equal(got[8], x[8].astype(np.float64))


def test_stale_view_raises_and_ops_see_writes(gpu):
    from oracle import spectra_oracle as orc
    from pypulsar_amd.formats.spectra import Spectra
    C, N = 16, 1024
    freqs = band(C)
    x = u8_data(C, N, 5)
    s = Spectra(freqs, DT, x)
    s.get_chan(0)[:] = 0.0
    ref = x.astype(np.float64)
    ref[0] = 0.0
    old = s.get_chan(1)
    s.dedisperse(20.0, padval=0, trim=True)
    with pytest.raises(RuntimeError):
        old[:] = 5.0                    # the Spectra changed since the view was taken
    want, _ = orc.dedisperse(ref, freqs, DT, 20.0, padval=0, trim=True)
    np.testing.assert_array_equal(s.data, want)
    # reading does not disturb anything
    assert float(np.asarray(s.data).sum()) == float(want.sum())


@pytest.mark.gpu
def test_two_open_views_both_write_through(gpu):
    """two views taken while the device data is unchanged share one
    host copy (the reference's get_chan views share self.data), so writing
    through the first and then the second keeps BOTH writes; a deep copy never
    shares the original's host copy."""
    import copy
    from pypulsar_amd.formats.spectra import Spectra
    C, N = 8, 512
    x = u8_data(C, N, 9)
    s = Spectra(band(C), DT, x)
    a = s.get_chan(0)
    b = s.get_chan(1)
    a[:] = 0.0
    b[:] = 0.0
    want = x.astype(np.float64)
    want[:2] = 0.0
    np.testing.assert_array_equal(s.data, want)
    d = copy.deepcopy(s)
    d.get_chan(2)[:] = 3.0
    np.testing.assert_array_equal(s.data, want)          # the original is untouched
    want_d = want.copy()
    want_d[2] = 3.0
    np.testing.assert_array_equal(d.data, want_d)
    sp = s.get_spectrum(5)
    sp[:] = 1.0
    want[:, 5] = 1.0
    np.testing.assert_array_equal(s.get_chan(3), want[3])
    np.testing.assert_array_equal(s.data, want)


@pytest.mark.gpu
def test_inplace_methods_and_float32_rounding_write_through(gpu):
    """in-place ndarray methods that skip __setitem__ / ufuncs
    (fill, put, sort) write through, and a float64 value that rounds in the
    float32 upload leaves the shared host copy equal to the device."""
    import torch
    from pypulsar_amd.formats.spectra import Spectra
    C, N = 4, 256
    x = u8_data(C, N, 11)
    s = Spectra(band(C), DT, x)
    s.get_chan(0).fill(2.0)
    np.testing.assert_array_equal(s._x[0].cpu().numpy(), np.full(N, 2.0, np.float32))
    s.get_chan(1).put([0, 3], [5.0, 6.0])
    assert s._x[1, 0].item() == 5.0 and s._x[1, 3].item() == 6.0
    c2 = s.get_chan(2)
    c2.sort()
    np.testing.assert_array_equal(s._x[2].cpu().numpy(), np.sort(x[2]).astype(np.float32))
    v = 0.1  # not a float32 value
    s.get_chan(3)[:] = v
    host = s.data
    assert host[3, 0] == np.float64(np.float32(v))
    np.testing.assert_array_equal(host, s._x.to(torch.float64).cpu().numpy())
