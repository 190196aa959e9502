"""CPU tests of the single-pulse search definition (oracle/search_oracle.py)
and of the host-side candidate handling of pypulsar_amd/search.py.  The
reference holds no search (boxcar = Pulse.smooth, formats/pulse.py:217-241):
these are known-answer tests of the definition, PRESTO parity unpinned."""
import numpy as np

from oracle import search_oracle as so

WIDTHS = (1, 2, 3, 4, 6, 9, 14, 20, 30)


def noise(D, n, seed):
    return np.random.default_rng(seed).normal(0.0, 1.0, (D, n))


def test_boxcar_snr_direct():
    z = noise(3, 200, 0)
    for w in (1, 5, 17):
        s = so.boxcar_snr(z, w)
        assert s.shape == (3, 200 - w + 1)
        for t in (0, 50, 200 - w):
            np.testing.assert_allclose(s[:, t], z[:, t:t + w].sum(axis=1) / np.sqrt(w), rtol=1e-12)


def test_normalise_chunks():
    x = np.concatenate([noise(1, 1000, 1) * 3 + 10, noise(1, 500, 2) * 0.5 - 4,
                        np.full((1, 7), 5.0)], axis=1)
    z = so.normalise(x, 500)
    for k in range(3):
        seg = z[0, k * 500:(k + 1) * 500]
        assert abs(seg.mean()) < 1e-12 and abs(seg.std() - 1) < 1e-12
    np.testing.assert_array_equal(z[0, 1500:], 0.0)  # constant short tail: std 0 -> 0


def test_known_pulses_found():
    D, n, L = 6, 5000, 1000
    x = noise(D, n, 3)
    inj = [(1, 700, 6, 5.0), (4, 3000, 20, 3.0), (5, 4990, 1, 12.0)]
    for d, t, w, a in inj:
        x[d, t:t + w] += a
    cands, margin = so.search(x, WIDTHS, 6.0, L)
    got = {(d, t // 1024): (t, w, s) for d, t, w, s in cands}
    for d, t, w, a in inj:
        t_, w_, s = got[(d, t // 1024)]
        assert abs(t_ - t) <= w and s > 6.0
    assert len(cands) == len(inj)
    assert all(m >= 0 for m in margin)


def test_tie_breaks_smallest_width_then_start():
    # a single spike: widths 1 gives snr = z; w=2 gives (z + z') / sqrt2, lower
    x = np.zeros((1, 2048))
    x[0, ::2] = 1.0
    x[0, 1::2] = -1.0
    x[0, 100] = 50.0
    cands, _ = so.search(x, (1, 2), 3.0, 2048)
    assert cands[0][1] == 100 and cands[0][2] == 1


def test_records_roundtrip(tmp_path):
    from pypulsar_amd import search
    raw = np.array([[2, 30, 4, 0], [0, 10, 1, 0]], dtype=np.int32)
    raw[:, 3] = np.array([7.5, 9.25], dtype=np.float32).view(np.int32)
    rec = search.to_records(raw, dms=[0.0, 5.0, 10.0], dt=1e-3, t0=100, starttime=2.0)
    assert list(rec["row"]) == [0, 2] and list(rec["Sample"]) == [110, 130]
    np.testing.assert_allclose(rec["Time"], [2.11, 2.13])
    np.testing.assert_allclose(rec["Sigma"], [9.25, 7.5])
    fn = str(tmp_path / "x.singlepulse")
    search.write_singlepulse(rec, fn)
    back = search.read_singlepulse(fn)
    np.testing.assert_allclose(back["DM"], rec["DM"])
    assert list(back["Sample"]) == [110, 130] and list(back["Downfact"]) == [1, 4]
    m = search.merge([rec[1:], None, rec[:1]])
    assert list(m["DM"]) == [0.0, 10.0]


def test_widths_validation():
    import pytest
    from pypulsar_amd import search
    with pytest.raises(AssertionError):
        search._widths([3, 2])
    with pytest.raises(AssertionError):
        search._widths([0, 1])
    with pytest.raises(AssertionError):
        search._widths(list(range(1, 40)))


def _golden_pulse():
    import os
    return np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                "golden_pulse.npz"), allow_pickle=False)


def test_boxcar_pinned_to_reference_pulse_smooth():
    """The search's boxcar (so.boxcar_snr) == the reference's Pulse.smooth
    (formats/pulse.py:217-241, run by tests/golden/make_golden_pulse.py) on
    every start whose boxcar lies inside the row: Pulse.smooth's output at
    t + w//2 is sum(z[t:t+w]) * float32(1/sqrt(w)) (convolve 'same' centres
    the top-hat there; the wrap padding only reaches the edges).  Tolerance:
    1e-6 relative -- the reference's kernel is float32(1/sqrt(w))."""
    g = _golden_pulse()
    z = g["z"]
    n = z.shape[1]
    for w in g["widths"]:
        w = int(w)
        ref = g["smooth_w%d" % w][:, w // 2:w // 2 + n - w + 1]
        got = so.boxcar_snr(z, w)
        assert got.shape == ref.shape
        np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-9 * np.abs(ref).max())


def test_downsample_pinned_to_reference_pulse_downsample():
    """Pulse.downsample (pulse.py:177-195, py2 division restored) == the
    oracle's Spectra.downsample restatement on one series (co-adds of f
    adjacent bins), bit for bit."""
    from oracle import spectra_oracle as orc
    g = _golden_pulse()
    x = g["ds_x"]
    for f in (1, 2, 3, 4, 8, 16):
        got, _ = orc.downsample(x, 64e-6, f)
        np.testing.assert_array_equal(got, g["ds_f%d" % f])
