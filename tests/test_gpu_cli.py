"""The drop-in CLIs on the GPU: zero_dm_filter, mockspecfil2subbands and
waterfaller (bin/*.py of the reference) end to end on synthetic filterbanks,
checked against the oracle restatement of the reference's per-spectrum /
per-channel loops."""
import os

import numpy as np
import pytest

from conftest import band, rel_err, u8_data
from oracle import spectra_oracle as orc

pytestmark = pytest.mark.gpu
DT = 64e-6


def _fil(tmp_path, x_tc, nbits=8, C=None, foff=None, name="in.fil"):
    from pypulsar_amd.formats import filterbank as fbm
    from pypulsar_amd.formats import sigproc
    C = x_tc.shape[1]
    foff = -300.0 / C if foff is None else foff
    params, hdr = sigproc.make_header(C, nbits, DT, 1550.0 + foff / 2, foff,
                                      src_raj=123456.789, src_dej=-123456.5)
    fn = str(tmp_path / name)
    fbm.write_filterbank(fn, params, hdr, x_tc)
    return fn


@pytest.mark.parametrize("dtype", [np.uint8, np.uint16, np.float32])
def test_zero_dm_filter_cli(gpu, tmp_path, dtype):
    from pypulsar_amd.bin import zero_dm_filter as z
    from pypulsar_amd.formats import filterbank as fbm
    rng = np.random.default_rng(3)
    nbits = {np.uint8: 8, np.uint16: 16, np.float32: 32}[dtype]
    if dtype == np.float32:
        x = rng.normal(0, 5, (5000, 40)).astype(dtype)
    else:
        x = rng.integers(0, np.iinfo(dtype).max, (5000, 40)).astype(dtype)
    fn = _fil(tmp_path, x, nbits)
    out = str(tmp_path / "out.fil")
    assert z.main(["-o", out, fn]) == 0
    fb = fbm.filterbank(out)
    got = fb.read_all_samples().reshape(-1, 40)
    want = orc.zero_dm_block(x)
    assert got.dtype == dtype and got.shape == x.shape
    if dtype == np.float32:
        assert rel_err(got, want) <= 1e-5
    else:
        np.testing.assert_array_equal(got, want)
    assert fb.header_params == fbm.filterbank(fn).header_params


@pytest.mark.parametrize("foff_sign", [-1, 1])
@pytest.mark.parametrize("all_samples", [False, True])
def test_mockspec_cli(gpu, tmp_path, foff_sign, all_samples):
    from pypulsar_amd.bin import mockspecfil2subbands as m
    C, N = 24, 3 * 4096 + 1000
    x = u8_data(C, N, 9).T.copy()  # [N, C]
    fn = _fil(tmp_path, x, foff=foff_sign * 2.0)
    outname = str(tmp_path / "sb")
    args = ["-o", outname, fn] + (["--all-samples"] if all_samples else [])
    assert m.main(args) == 0
    nw = N if all_samples else (N // 4096 - 1) * 4096 + N % 4096
    for k in range(C):
        j = k if foff_sign > 0 else C - 1 - k  # reversed numbering when foff < 0
        got = np.fromfile("%s.sub%04d" % (outname, k), dtype=np.uint8)
        np.testing.assert_array_equal(got, x[:nw, j])
    inf = open(outname + ".sub.inf").read()
    assert "Number of bins in the time series      =  %d" % N in inf
    assert "12:34:56.789" in inf and "-12:34:56.5" in inf
    assert "Number of channels                     =  %d" % C in inf


def test_waterfaller_cli(gpu, tmp_path):
    from pypulsar_amd.bin import waterfaller as w
    C, N = 64, 12000  # 3000 bins + the 150 pc/cc sweep (6201 bins at 1250 MHz)
    x = u8_data(C, N, 13)
    fn = _fil(tmp_path, x.T.copy())
    png = str(tmp_path / "wf.png")
    assert w.main(["-T", "0.01", "-n", "3000", "-d", "150", "--subdm", "150", "-s", "16",
                   "--downsamp", "2", "--width-bins", "3", "--sweep-dm", "150",
                   "--outfile", png, fn]) == 0
    assert os.path.getsize(png) > 1000
    # the device pipeline equals the oracle composition of waterfaller.py:103-127
    from pypulsar_amd.formats import filterbank as fbm
    opts = type("O", (), dict(dm=150.0, start=0.01, duration=None, nbins=3000, maskfile=None,
                              width_bins=3, downsamp=2, nsub=16, subdm=150.0, scaleindep=False))
    data = w.run(fn, opts)
    fb = fbm.filterbank(fn)
    start = int(np.round(0.01 / DT))
    nb = 3000 + int(np.round(orc.delay_from_DM(150.0, fb.freqs.min()) / DT))
    d = x[:, start:start + nb].astype(np.float64)
    d, f = orc.subband(d, fb.freqs, DT, 16, 150.0, padval="mean")
    d, _ = orc.dedisperse(d, f, DT, 150.0, padval="mean", trim=True)
    d, _ = orc.downsample(d, DT, 2)
    d = orc.smooth(orc.scaled(d), 3, "mean")
    assert data.data.shape == d.shape
    assert rel_err(data.data, d) <= 1e-5


def test_waterfaller_mask(gpu, tmp_path):
    """--mask: the rfifind mask of the span (get_mask, waterfaller.py:28-48)
    applied with masked(..., 'median-mid80') before the chain
    (waterfaller.py:92-99), against the oracle composition."""
    from pypulsar_amd.bin import waterfaller as w
    from pypulsar_amd.formats import filterbank as fbm
    from pypulsar_amd.formats import rfifind as rf
    C, N, ppi = 64, 12000, 1000
    x = u8_data(C, N, 21)
    fn = _fil(tmp_path, x.T.copy())
    rng = np.random.default_rng(5)
    per = [np.sort(rng.choice(C, size=int(rng.integers(0, 12)), replace=False))
           for _ in range(N // ppi)]
    per[3] = np.arange(C)  # a fully zapped interval
    mfn = str(tmp_path / "in_rfifind.mask")
    rf.write_mask(mfn, C, ppi, per)
    png = str(tmp_path / "wf.png")
    assert w.main(["-T", "0.01", "-n", "3000", "-d", "150", "-s", "16", "--mask", mfn,
                   "--outfile", png, fn]) == 0
    opts = type("O", (), dict(dm=150.0, start=0.01, duration=None, nbins=3000, maskfile=mfn,
                              width_bins=1, downsamp=1, nsub=16, subdm=150.0, scaleindep=False))
    data = w.run(fn, opts)
    fb = fbm.filterbank(fn)
    start = int(np.round(0.01 / DT))
    nb = 3000 + int(np.round(orc.delay_from_DM(150.0, fb.freqs.min()) / DT))
    d = x[:, start:start + nb].astype(np.float64)
    mask = np.zeros_like(d, dtype=bool)
    for j in range(nb):
        mask[per[(start + j) // ppi], j] = True
    d = orc.masked(d, mask, "median-mid80")
    d, f = orc.subband(d, fb.freqs, DT, 16, 150.0, padval="mean")
    d, _ = orc.dedisperse(d, f, DT, 150.0, padval="mean", trim=True)
    d = orc.scaled(d)
    assert data.data.shape == d.shape
    assert rel_err(data.data, d) <= 1e-5


def test_waterfaller_psrfits(gpu, tmp_path):
    """waterfaller.py on a PSRFITS file (waterfaller.py:58-59 opens .fits with
    psrfits.PsrfitsFile): same pipeline result as on a filterbank holding the
    same spectra (scales 1, offsets 0, weights 1; descending band)."""
    from pypulsar_amd.bin import waterfaller as w
    from pypulsar_amd.formats.psrfits import write_search_psrfits
    C, nsblk, nsub = 64, 1000, 12
    x = u8_data(C, nsblk * nsub, 21)                     # [C, N]
    fil = _fil(tmp_path, x.T.copy())
    from pypulsar_amd.formats import filterbank as fbm
    freqs = fbm.filterbank(fil).freqs                    # descending, as written
    fits_fn = str(tmp_path / "wf.fits")
    write_search_psrfits(fits_fn, x.T.reshape(nsub, nsblk, C), freqs, DT, 8)
    png = str(tmp_path / "wf2.png")
    assert w.main(["-T", "0.01", "-n", "2000", "-d", "100", "-s", "16", "--outfile", png,
                   fits_fn]) == 0
    assert os.path.getsize(png) > 1000
    opts = type("O", (), dict(dm=100.0, start=0.01, duration=None, nbins=2000, maskfile=None,
                              width_bins=1, downsamp=1, nsub=16, subdm=100.0, scaleindep=False))
    a = w.run(fits_fn, opts).data
    b = w.run(fil, opts).data
    assert a.shape == b.shape
    np.testing.assert_array_equal(a, b)


def test_frb_search_cli(gpu, tmp_path):
    """frb_search.py end to end: a burst dispersed at DM 40 in a 3-block
    8-bit filterbank comes out of the .singlepulse file at its DM and time."""
    from pypulsar_amd.bin import frb_search as fs
    from pypulsar_amd.delays import delay_from_DM
    from pypulsar_amd.search import read_singlepulse
    C, N, block = 128, 3 * 8192, 8192
    x = u8_data(C, N, 31).astype(np.int32).T.copy()     # [N, C] file order
    fn0 = _fil(tmp_path, x.astype(np.uint8))
    from pypulsar_amd.formats import filterbank as fbm
    freqs = fbm.filterbank(fn0).freqs
    bins = np.round((delay_from_DM(40.0, freqs) - delay_from_DM(40.0, freqs.max())) / DT)
    t_arr = 9000
    for c in range(C):
        x[t_arr + int(bins[c]):t_arr + int(bins[c]) + 8, c] += 30
    fn = _fil(tmp_path, np.clip(x, 0, 255).astype(np.uint8), name="burst.fil")
    out = str(tmp_path / "burst.singlepulse")
    assert fs.main(["--lodm", "0", "--hidm", "80", "--numdms", "81", "--downsamp", "2",
                    "--block", str(block), "-t", "8", "-o", out, fn]) == 0
    cands = read_singlepulse(out)
    assert len(cands) >= 1
    best = cands[np.argmax(cands["Sigma"])]
    assert abs(best["DM"] - 40.0) <= 2.0
    assert abs(best["Time"] - t_arr * DT) <= 16 * DT
