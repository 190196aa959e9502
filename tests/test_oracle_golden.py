"""Pin the oracle (oracle/spectra_oracle.py) to the golden fixtures that the
reference itself produced (tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest

from oracle import spectra_oracle as orc
from conftest import PADS

DT = 64e-6


@pytest.mark.parametrize("C", [64, 1024, 4096])
@pytest.mark.parametrize("tag", ["desc", "asc"])
def test_bins_bit_exact(golden, C, tag):
    key = "bins_C%d_%s" % (C, tag)
    freqs = golden[key + "_freqs"]
    for i, dm in enumerate(golden["bins_dms"]):
        assert np.array_equal(orc.dedisperse_bins(dm, 0.0, freqs, DT), golden[key][i])


def test_bins_grid(golden):
    from conftest import band
    freqs = band(1024)
    tab = orc.sweep_table(golden["bins_grid_dms"], freqs, DT)
    assert np.array_equal(tab, golden["bins_grid"])


@pytest.mark.parametrize("tag", ["desc", "asc"])
@pytest.mark.parametrize("pi", range(5))
@pytest.mark.parametrize("trim", [False, True])
def test_dedisperse(golden, tag, pi, trim):
    x = golden["dd_x"].astype(np.float64)
    freqs = golden["dd_freqs_" + tag]
    pad = PADS[pi]
    for dm in (100, 3000):
        got, _ = orc.dedisperse(x, freqs, DT, float(dm), padval=pad, trim=trim)
        want = golden["dd_%s_p%d_t%d_dm%d" % (tag, pi, int(trim), dm)]
        assert got.shape == want.shape
        np.testing.assert_allclose(got, want, rtol=0, atol=1e-9)
    a, cur = orc.dedisperse(x, freqs, DT, 100.0, padval=pad)
    got, _ = orc.dedisperse(a, freqs, DT, 50.0, cur_dm=cur, padval=pad, trim=trim)
    want = golden["dd2_%s_p%d_t%d" % (tag, pi, int(trim))]
    assert got.shape == want.shape
    np.testing.assert_allclose(got, want, rtol=0, atol=1e-9)


@pytest.mark.parametrize("tag", ["desc", "asc"])
@pytest.mark.parametrize("nsub", [1, 8, 32])
@pytest.mark.parametrize("si", range(4))
@pytest.mark.parametrize("pi", range(2))
def test_subband(golden, golden_meta, tag, nsub, si, pi):
    x = golden["sb_x"].astype(np.float64)
    freqs = golden["sb_freqs_" + tag]
    subdm = golden_meta["subdms"][si]
    pad = [0, "mean"][pi]
    k = "sb_%s_n%d_s%d_p%d" % (tag, nsub, si, pi)
    got, f = orc.subband(x, freqs, DT, nsub, subdm, padval=pad)
    np.testing.assert_allclose(got, golden[k], rtol=0, atol=1e-9)
    assert np.array_equal(f, golden[k + "_freqs"])
    if subdm is not None:
        assert np.array_equal(orc.subband_bins(subdm, 0.0, freqs, DT, nsub), golden[k + "_bins"])


@pytest.mark.parametrize("tag", ["desc", "asc"])
def test_subband_then_dedisperse(golden, tag):
    x = golden["sb_x"].astype(np.float64)
    freqs = golden["sb_freqs_" + tag]
    s, f = orc.subband(x, freqs, DT, 8, 100.0, padval="mean")
    got, _ = orc.dedisperse(s, f, DT, 100.0, padval="mean", trim=True)
    np.testing.assert_allclose(got, golden["sbdd_" + tag], rtol=0, atol=1e-9)


@pytest.mark.parametrize("f", [1, 3, 4, 7, 8])
def test_downsample(golden, f):
    x = golden["ds_x"].astype(np.float64)
    got, dt = orc.downsample(x, DT, f)
    np.testing.assert_array_equal(got, golden["ds_f%d" % f])
    assert dt == float(golden["ds_f%d_dt" % f])
    assert got.shape[1] == int(golden["ds_f%d_n" % f])


def test_trim(golden):
    x = golden["ds_x"].astype(np.float64)
    d, n, st = orc.trim(x, 10, 1.0, DT)
    np.testing.assert_array_equal(d, golden["trim_pos"])
    assert [n, st] == list(golden["trim_pos_meta"])
    d, n, st = orc.trim(x, -10, 1.0, DT)
    np.testing.assert_array_equal(d, golden["trim_neg"])
    assert n == golden["trim_neg_meta"][0]
    assert st == pytest.approx(golden["trim_neg_meta"][1], abs=0)


@pytest.mark.parametrize("name", ["u8", "u16", "f32", "tie", "probe"])
def test_zero_dm(golden, name):
    inp = golden["zd_in_" + name]
    got = orc.zero_dm_block(inp)
    want = golden["zd_out_" + name]
    assert got.dtype == want.dtype
    np.testing.assert_array_equal(got, want)


def test_zero_dm_probe_vector(golden):
    # documented reference behaviour: uint8 wrap
    assert list(golden["zd_out_probe"][0]) == [188, 122, 22, 181]


def test_sweep_plane(golden):
    x = golden["sw_x"].astype(np.float64)
    freqs = golden["sw_freqs"]
    tab = orc.sweep_table(golden["sw_dms"], freqs, DT)
    plane = orc.sweep_plane(x, tab)
    np.testing.assert_array_equal(plane, golden["sw_plane"])
    # the common width is N - max bin; reference per-row lengths are >= it
    assert plane.shape[1] == min(golden["sw_lens"])


@pytest.mark.parametrize("pi", [0, 1])
def test_sweep_plane_full(golden, pi):
    x = golden["sw_x"].astype(np.float64)
    tab = orc.sweep_table(golden["sw_dms"], golden["sw_freqs"], DT)
    pad = [0, "mean"][pi]
    plane = orc.sweep_plane(x, tab, padval=pad, n_out=x.shape[1])
    np.testing.assert_allclose(plane, golden["sw_plane_full_p%d" % pi], rtol=1e-12, atol=1e-9)


def test_two_stage_sweep(golden, golden_meta):
    x = golden["sw_x"].astype(np.float64)
    freqs = golden["sw_freqs"]
    p = golden_meta["sw2"]
    sub, f = orc.subband(x, freqs, DT, p["nsub"], p["subDM"], padval=0)
    tab = orc.sweep_table(golden["sw2_dms"], f, DT)
    plane = orc.sweep_plane(sub, tab)
    np.testing.assert_array_equal(plane, golden["sw2_plane"])


def test_downsample_then_dedisperse(golden):
    x = golden["sw_x"].astype(np.float64)
    d, dt = orc.downsample(x, DT, 4)
    dd, _ = orc.dedisperse(d, golden["sw_freqs"], dt, 200.0, trim=True)
    np.testing.assert_array_equal(orc.channel_sum(dd), golden["dsdd_series"])


def test_sweep_rows_inside_equals_sweep_plane():
    """The fast pad-free row restatement equals the per-channel shifted sum."""
    from oracle import spectra_oracle as orc
    rng = np.random.default_rng(9)
    x = rng.integers(0, 256, size=(32, 700), dtype=np.uint8)
    foff = -300.0 / 32
    freqs = 1550.0 + foff / 2 + foff * np.arange(32)
    tab = orc.sweep_table(np.linspace(0, 30, 7), freqs, 64e-6)
    want = orc.sweep_plane(x.astype(np.float64), tab)
    np.testing.assert_array_equal(orc.sweep_rows_inside(x, tab, want.shape[1]), want)
