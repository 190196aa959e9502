"""GPU parity: every libpdd kernel, called through the C ABI (via the
pypulsar_amd Spectra / DMSweep / zero_dm wrappers), against the golden
fixtures and the oracle on the same seeded inputs.

Bar: bit-exact for integer data with integer pads, integer tables and
byte work; float32 results (mean pads, fractional data) within
max|gpu - ref| <= 1e-5 * max|ref| per array."""
import copy

import numpy as np
import pytest

from conftest import PADS, band, rel_err, u8_data
from oracle import spectra_oracle as orc

pytestmark = pytest.mark.gpu
DT = 64e-6
TOL = 1e-5


def exact_or_tol(got, want, exact):
    assert got.shape == want.shape, (got.shape, want.shape)
    if exact:
        np.testing.assert_array_equal(got, want)
    else:
        assert rel_err(got, want) <= TOL


@pytest.fixture(scope="module")
def S(gpu):
    from pypulsar_amd.formats.spectra import Spectra
    return Spectra


# ------------------------------------------------------------------ dedisperse
@pytest.mark.parametrize("tag", ["desc", "asc"])
@pytest.mark.parametrize("pi", range(5))
@pytest.mark.parametrize("trim", [False, True])
def test_dedisperse_golden(S, golden, tag, pi, trim):
    x = golden["dd_x"]
    freqs = golden["dd_freqs_" + tag]
    pad = PADS[pi]
    exact = pad != "mean"
    for dm in (100, 3000):
        s = S(freqs, DT, x)
        s.dedisperse(float(dm), padval=pad, trim=trim)
        want = golden["dd_%s_p%d_t%d_dm%d" % (tag, pi, int(trim), dm)]
        exact_or_tol(s.data, want, exact)
        # reference arithmetic: numspectra = N - ntrim even when ntrim > N
        assert s.dm == dm and (s.numspectra == want.shape[1] if want.shape[1] else s.numspectra <= 0)
    s = S(freqs, DT, x)
    s.dedisperse(100.0, padval=pad)
    s.dedisperse(50.0, padval=pad, trim=trim)  # negative shifts
    exact_or_tol(s.data, golden["dd2_%s_p%d_t%d" % (tag, pi, int(trim))], exact)


def test_dedisperse_f_order_input(S):
    # filterbank.get_spectra hands Spectra the transpose of an [N, C] block
    C, N = 96, 3000
    freqs = band(C)
    blk = np.ascontiguousarray(u8_data(C, N, 7).T)  # [N, C]
    s = S(freqs, DT, blk.T)
    assert s._raw8 is not None
    s.dedisperse(250.0, trim=True)
    want, _ = orc.dedisperse(blk.T.astype(np.float64), freqs, DT, 250.0, trim=True)
    np.testing.assert_array_equal(s.data, want)


@pytest.mark.parametrize("dtype", [np.uint16, np.float32, np.float64])
def test_constructor_dtypes(S, dtype):
    C, N = 33, 517
    x = (np.random.default_rng(1).random((C, N)) * 1000).astype(dtype)
    s = S(band(C), DT, x)
    np.testing.assert_array_equal(s.data, x.astype(np.float32).astype(np.float64))
    s2 = S(band(C), DT, np.asfortranarray(x))
    np.testing.assert_array_equal(s2.data, s.data)


# ------------------------------------------------------------------ subband
@pytest.mark.parametrize("tag", ["desc", "asc"])
@pytest.mark.parametrize("nsub", [1, 8, 32])
@pytest.mark.parametrize("si", range(4))
@pytest.mark.parametrize("pi", range(2))
def test_subband_golden(S, golden, golden_meta, tag, nsub, si, pi):
    x = golden["sb_x"]
    freqs = golden["sb_freqs_" + tag]
    subdm = golden_meta["subdms"][si]
    pad = [0, "mean"][pi]
    k = "sb_%s_n%d_s%d_p%d" % (tag, nsub, si, pi)
    s = S(freqs, DT, x)
    s.subband(nsub, subdm, padval=pad)
    exact_or_tol(s.data, golden[k], pad != "mean")
    assert np.array_equal(s.freqs, golden[k + "_freqs"]) and s.numchans == nsub and s.dm == 0


@pytest.mark.parametrize("tag", ["desc", "asc"])
def test_waterfaller_chain(S, golden, tag):
    s = S(golden["sb_freqs_" + tag], DT, golden["sb_x"])
    s.subband(8, 100.0, padval="mean")
    s.dedisperse(100.0, padval="mean", trim=True)
    exact_or_tol(s.data, golden["sbdd_" + tag], False)


def test_subband_rotate_and_asserts(S):
    C, N = 64, 700
    freqs = band(C, False)
    x = u8_data(C, N, 11)
    s = S(freqs, DT, x)
    s.subband(4, 300.0, padval="rotate")
    want, _ = orc.subband(x.astype(np.float64), freqs, DT, 4, 300.0, padval="rotate")
    np.testing.assert_array_equal(s.data, want)
    with pytest.raises(AssertionError):
        S(freqs, DT, x).subband(5)
    with pytest.raises(AssertionError):
        S(freqs, DT, x).subband(4, -1.0)
    with pytest.raises(AssertionError):
        S(freqs, DT, x).dedisperse(-1.0)


# ------------------------------------------------------------------ downsample / trim
@pytest.mark.parametrize("f", [1, 3, 4, 7, 8])
def test_downsample_golden(S, golden, f):
    s = S(band(8), DT, golden["ds_x"])
    s.downsample(f)
    np.testing.assert_array_equal(s.data, golden["ds_f%d" % f])
    assert s.numspectra == int(golden["ds_f%d_n" % f]) and s.dt == float(golden["ds_f%d_dt" % f])


def test_downsample_no_trim_assert(S, golden):
    s = S(band(8), DT, golden["ds_x"])  # N = 1000
    with pytest.raises(AssertionError):
        s.downsample(3, trim=False)
    s.downsample(8, trim=False)
    assert s.numspectra == 125


def test_trim_golden(S, golden):
    s = S(band(8), DT, golden["ds_x"], starttime=1.0)
    s.trim(10)
    np.testing.assert_array_equal(s.data, golden["trim_pos"])
    assert [s.numspectra, s.starttime] == list(golden["trim_pos_meta"])
    s = S(band(8), DT, golden["ds_x"], starttime=1.0)
    s.trim(-10)
    np.testing.assert_array_equal(s.data, golden["trim_neg"])
    assert s.numspectra == golden["trim_neg_meta"][0]
    with pytest.raises(AssertionError):
        s.trim(10 ** 6)


def test_downsample_then_dedisperse(S, golden):
    s = S(golden["sw_freqs"], DT, golden["sw_x"])
    s.downsample(4)
    s.dedisperse(200.0, trim=True)
    np.testing.assert_array_equal(s.sum_channels().cpu().numpy(), golden["dsdd_series"])


# ------------------------------------------------------------------ series / stats
@pytest.mark.parametrize("pad", PADS)
def test_dedispersed_series(S, pad):
    C, N = 200, 5000
    freqs = band(C)
    x = u8_data(C, N, 12)
    s = S(freqs, DT, x)
    for dm, trim in ((0.0, True), (75.0, True), (75.0, False), (900.0, False)):
        got = s.dedispersed_series(dm, padval=pad, trim=trim).cpu().numpy()
        d, _ = orc.dedisperse(x.astype(np.float64), freqs, DT, dm, padval=pad, trim=trim)
        want = orc.channel_sum(d)
        exact_or_tol(got.astype(np.float64), want, pad != "mean")
    # the fused series leaves the Spectra untouched
    np.testing.assert_array_equal(s.data, x.astype(np.float64))


def test_channel_median_exact(S):
    import torch
    from pypulsar_amd import _lib
    rng = np.random.default_rng(3)
    for N in (1, 2, 7, 1000, 4097):
        x = rng.normal(size=(9, N)).astype(np.float32)
        x[0] = 5.0  # ties
        x[1, : N // 2] = -0.0
        t = torch.from_numpy(x).cuda()
        out = torch.empty(9, device="cuda")
        _lib.call("pdd_channel_stats", _lib.ptr(t), 9, N, N, _lib.STAT_MEDIAN, _lib.ptr(out),
                  _lib.stream_ptr())
        want = np.median(x.astype(np.float64), axis=1)
        np.testing.assert_allclose(out.cpu().numpy(), want, rtol=1e-7, atol=0)


# ------------------------------------------------------------------ zero-DM
@pytest.mark.parametrize("name", ["u8", "u16", "f32", "tie", "probe"])
@pytest.mark.parametrize("layout", ["time", "chan"])
def test_zero_dm_golden(gpu, golden, name, layout):
    from pypulsar_amd.zero_dm import zero_dm
    inp = golden["zd_in_" + name]
    want = golden["zd_out_" + name]
    if layout == "time":
        got = zero_dm(inp, "time")
    else:
        got = zero_dm(np.ascontiguousarray(inp.T), "chan").T
    assert got.dtype == want.dtype
    if inp.dtype == np.float32:
        assert rel_err(got, want) <= TOL
    else:
        np.testing.assert_array_equal(got, want)


def test_zero_dm_large_u8(gpu):
    import torch
    from pypulsar_amd.zero_dm import zero_dm
    blk = np.random.default_rng(9).integers(0, 256, size=(3000, 4096), dtype=np.uint8)
    got = zero_dm(torch.from_numpy(blk).cuda(), "time").cpu().numpy()
    np.testing.assert_array_equal(got, orc.zero_dm_block(blk))


# ------------------------------------------------------------------ corner turn
@pytest.mark.parametrize("dt_", [np.uint8, np.uint16, np.float32])
def test_corner_turn(gpu, dt_):
    import torch
    from pypulsar_amd import _lib
    nspec, nchan = 1000, 333
    a = (np.random.default_rng(2).random((nspec, nchan)) * 200).astype(dt_)
    code = {np.uint8: _lib.U8, np.uint16: _lib.U16, np.float32: _lib.F32}[dt_]
    src = torch.from_numpy(a.view(np.int16) if dt_ == np.uint16 else a).cuda()
    out = torch.empty((nchan, nspec), dtype=torch.float32, device="cuda")
    _lib.call("pdd_corner_turn", _lib.ptr(src), code, nspec, nchan, nchan, _lib.ptr(out),
              _lib.F32, nspec, _lib.stream_ptr())
    np.testing.assert_array_equal(out.cpu().numpy(), a.T.astype(np.float32))
    if dt_ == np.uint8:
        o8 = torch.empty((nchan, nspec), dtype=torch.uint8, device="cuda")
        _lib.call("pdd_corner_turn", _lib.ptr(src), code, nspec, nchan, nchan, _lib.ptr(o8),
                  _lib.U8, nspec, _lib.stream_ptr())
        np.testing.assert_array_equal(o8.cpu().numpy(), a.T)


@pytest.mark.parametrize("nspec,nchan", [(1007, 400), (128, 64), (4096, 4096), (17, 16)])
def test_corner_turn_b8_vector(gpu, nspec, nchan):
    """The 16-byte 8-bit raw corner turn (aligned rows): tiles of 128 spectra
    x 64 channels, partial tiles at both edges, a bytewise nspec tail, and no
    write past nspec in a padded output row."""
    import torch
    from pypulsar_amd import _lib
    a = np.random.default_rng(5).integers(0, 256, (nspec, nchan), dtype=np.uint8)
    src = torch.from_numpy(a).cuda()
    ld_out = (nspec + 15) // 16 * 16 + 16
    o8 = torch.full((nchan, ld_out), 7, dtype=torch.uint8, device="cuda")
    _lib.call("pdd_corner_turn", _lib.ptr(src), _lib.U8, nspec, nchan, nchan, _lib.ptr(o8),
              _lib.U8, ld_out, _lib.stream_ptr())
    got = o8.cpu().numpy()
    np.testing.assert_array_equal(got[:, :nspec], a.T)
    assert (got[:, nspec:] == 7).all()


# ------------------------------------------------------------------ sweep
@pytest.mark.parametrize("dtype", ["f32", "u8"])
def test_sweep_golden(gpu, golden, dtype):
    import torch
    from pypulsar_amd.sweep import DMSweep
    x = golden["sw_x"]
    sw = DMSweep(golden["sw_dms"], golden["sw_freqs"], DT, dtype=dtype)
    xd = torch.from_numpy(x).cuda()
    plane = sw(xd.float() if dtype == "f32" else xd).cpu().numpy()
    np.testing.assert_array_equal(plane.astype(np.float64), golden["sw_plane"])
    for pi, pad in enumerate([0, "mean"]):
        if dtype == "u8" and pad == "mean":
            continue
        full = sw(xd.float() if dtype == "f32" else xd, padval=pad, trim=False).cpu().numpy()
        exact_or_tol(full.astype(np.float64), golden["sw_plane_full_p%d" % pi], pad == 0)


@pytest.mark.parametrize("dtype", ["f32", "u8"])
@pytest.mark.parametrize("pad", [0, 7, "rotate", 2.5, "median"])
def test_sweep_pads_and_negative_shifts(gpu, dtype, pad):
    """trim=False rows use every pad mode; cur_dm > dm gives negative shifts."""
    import torch
    from pypulsar_amd.sweep import DMSweep
    C, N = 48, 3000
    freqs = band(C)
    x = u8_data(C, N, 21)
    dms = np.linspace(0.0, 120.0, 37)
    for cur in (0.0, 60.0):
        sw = DMSweep(dms, freqs, DT, cur_dm=cur, dtype=dtype)
        xd = torch.from_numpy(x).cuda()
        got = sw(xd.float() if dtype == "f32" else xd, padval=pad, trim=False).cpu().numpy()
        tab = orc.sweep_table(dms, freqs, DT, cur_dm=cur)
        want = orc.sweep_plane(x.astype(np.float64), tab, padval=pad, n_out=N)
        exact_or_tol(got.astype(np.float64), want, True)  # integer data, .5 pads: exact
        sw.close()


@pytest.mark.parametrize("dtype", ["f32", "u8"])
def test_sweep_spectra_and_twostage(S, golden, golden_meta, dtype):
    x = golden["sw_x"]
    freqs = golden["sw_freqs"]
    s = S(freqs, DT, x if dtype == "u8" else x.astype(np.float32))
    plane = s.sweep(golden["sw_dms"]).cpu().numpy()
    np.testing.assert_array_equal(plane.astype(np.float64), golden["sw_plane"])
    p = golden_meta["sw2"]
    s.subband(p["nsub"], p["subDM"], padval=0)
    plane2 = s.sweep(golden["sw2_dms"]).cpu().numpy()
    np.testing.assert_array_equal(plane2.astype(np.float64), golden["sw2_plane"])


def test_sweep_float_data(gpu):
    import torch
    from pypulsar_amd.sweep import DMSweep
    C, N = 256, 6000
    freqs = band(C)
    x = np.random.default_rng(5).normal(size=(C, N)).astype(np.float32)
    dms = np.linspace(5.0, 400.0, 70)
    sw = DMSweep(dms, freqs, DT)
    got = sw(torch.from_numpy(x).cuda()).cpu().numpy().astype(np.float64)
    want = orc.sweep_plane(x.astype(np.float64), orc.sweep_table(dms, freqs, DT))
    assert got.shape == want.shape
    for d in range(len(dms)):
        assert rel_err(got[d], want[d]) <= TOL


def test_sweep_sparse_grid_and_odd_sizes(gpu):
    """Sparse DM grid (wide LDS spans -> smaller tile variants), D not a
    multiple of the DM block, N not a multiple of the time tile."""
    import torch
    from pypulsar_amd.sweep import DMSweep
    C, N = 37, 50000
    freqs = band(C)
    x = u8_data(C, N, 8)
    for dms in (np.array([0.0, 1500.0, 3000.0]), np.arange(0.0, 2000.0, 97.0),
                np.array([123.4])):
        for dtype in ("f32", "u8"):
            sw = DMSweep(dms, freqs, DT, dtype=dtype)
            xd = torch.from_numpy(x).cuda()
            got = sw(xd.float() if dtype == "f32" else xd).cpu().numpy()
            want = orc.sweep_plane(x.astype(np.float64), orc.sweep_table(dms, freqs, DT))
            np.testing.assert_array_equal(got.astype(np.float64), want)
            sw.close()


def test_sweep_large_properties(gpu):
    """Config-2 channel count at reduced length: rows equal the fused single-DM
    series (independent kernel), and the u8 and f32 kernels agree bit for bit."""
    import torch
    from pypulsar_amd.formats.spectra import Spectra
    from pypulsar_amd.sweep import DMSweep
    C, N = 1024, 1 << 17
    freqs = band(C)
    x = u8_data(C, N, 13)
    dms = np.linspace(0.0, 1000.0, 1024)
    xd = torch.from_numpy(x).cuda()
    p32 = DMSweep(dms, freqs, DT, dtype="f32")(xd.float())
    p8 = DMSweep(dms, freqs, DT, dtype="u8")(xd)
    assert torch.equal(p32, p8)
    s = Spectra(freqs, DT, x)
    n_out = p32.shape[1]
    for d in (0, 1, 511, 1023):
        ser = s.dedispersed_series(dms[d], trim=True)[:n_out]
        assert torch.equal(ser, p32[d])
    # checksum of checksums against the oracle on a subsample of rows
    tab = orc.sweep_table(dms[::255], freqs, DT)
    want = orc.sweep_plane(x.astype(np.float64), tab, n_out=n_out)
    np.testing.assert_array_equal(p32[::255].cpu().numpy().astype(np.float64), want)


def test_execute_ddplan(S):
    from pypulsar_amd.sweep import execute_plan
    from pypulsar_amd.utils.ddplan import Observation
    C, N = 64, 8192
    freqs = band(C)
    x = u8_data(C, N, 17)
    obs = Observation(DT, 1400.0, 300.0, C)
    for nsub, res in ((0, 0.0), (8, 1.0)):
        plan = obs.gen_ddplan(0.0, 120.0, nsub, res)
        s = S(freqs, DT, x)
        res_ = execute_plan(s, plan)
        for step, outs in res_:
            xd, dt = orc.downsample(x.astype(np.float64), DT, step.downsamp)
            for (subdm, dms), (dms2, plane) in zip(step.subband_calls(), outs):
                assert np.array_equal(dms, dms2)
                if subdm is None:
                    src, f = xd, freqs
                else:
                    src, f = orc.subband(xd, freqs, dt, nsub, subdm, padval=0)
                want = orc.sweep_plane(src, orc.sweep_table(dms, f, dt))
                np.testing.assert_array_equal(plane.cpu().numpy().astype(np.float64), want)


def test_deepcopy_independent(S):
    x = u8_data(16, 100, 1)
    s = S(band(16), DT, x)
    t = copy.deepcopy(s)
    t.dedisperse(500.0)
    np.testing.assert_array_equal(s.data, x.astype(np.float64))


# Every tiling the plan can choose, reached by a grid whose per-trial-block
# shift span forces it (pdd_sweep.hip kF32Variants / kU8Variants, best first),
# each checked against the oracle.  The dDM of each rung comes from the
# plan-selection model tests/plan_model.py (asserted equal to the library's
# choice): rung i selects candidate i.
LADDER = {"f32": [2.0, 8.0, 15.0, 40.0],
          "u8": [1.0, 3.0, 8.0, 15.0, 40.0]}


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["f32", "u8"])
def test_sweep_variant_ladder(gpu, dtype):
    import torch
    import plan_model
    from pypulsar_amd.sweep import DMSweep
    C, N, D = 32, 49152, 64
    freqs = band(C)
    x = u8_data(C, N, 21)
    xd = torch.from_numpy(x).cuda()
    if dtype == "f32":
        xd = xd.float()
    code = 1 if dtype == "u8" else 0
    for want_v, ddm in enumerate(LADDER[dtype]):
        dms = np.arange(D) * ddm
        tab = orc.sweep_table(dms, freqs, DT)
        assert plan_model.choose(tab, dtype) == want_v
        sw = DMSweep(dms, freqs, DT, dtype=dtype)
        v = sw.info(code)["variant"]
        assert v == want_v, "dDM %g chose variant %d, expected %d" % (ddm, v, want_v)
        plane = sw(xd).cpu().numpy().astype(np.float64)
        want = orc.sweep_plane(x.astype(np.float64), tab)
        np.testing.assert_array_equal(plane, want, err_msg="dDM %g (variant %d)" % (ddm, v))
        sw.close()


@pytest.mark.gpu
@pytest.mark.parametrize("pad", [0, 7, "rotate"])
def test_grouped_u8_sweep(gpu, pad):
    """Grouped 8-bit sweep (u16-eighths VALU kernel, kU8Variants[0]): two
    channel groups with their own tables, against per-group oracle planes."""
    import torch
    from pypulsar_amd import _lib
    from pypulsar_amd.sweep import GroupedSweep
    C, N, G = 24, 6000, 2
    freqs = band(C)
    x = u8_data(G * C, N, 22)
    tabs = np.stack([orc.sweep_table(np.linspace(0, 30, 10), freqs, DT),
                     orc.sweep_table(np.linspace(5, 60, 10), freqs, DT)])
    gs = GroupedSweep(tabs, "u8")
    n_out = N  # untrimmed: the last columns read pads / wrapped samples
    out = torch.zeros((G * 10, n_out), dtype=torch.float32, device="cuda")
    if pad == "rotate":
        mode, pv = _lib.PAD_ROTATE, None
    else:
        mode, pv = _lib.PAD_VALUE, torch.full((G * C,), float(pad), device="cuda")
    gs(torch.from_numpy(x).cuda(), n_out, out, row_g=10, row_d=1, pad_mode=mode, padvals=pv)
    got = out.cpu().numpy().astype(np.float64)
    for g in range(G):
        want = orc.sweep_plane(x[g * C:(g + 1) * C].astype(np.float64), tabs[g], padval=pad,
                               n_out=n_out)
        np.testing.assert_array_equal(got[g * 10:(g + 1) * 10], want)
    gs.close()


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["u8", "f32"])
def test_sweep_pieces_layout_and_offset(gpu, dtype):
    """pdd_sweep_execute_ex: a block in the all-gathered "pieces" layout
    [N/P][C][P] and a column offset give exactly those columns of the
    channel-major one-shot plane (the DM-sharded path's input)."""
    import torch
    from pypulsar_amd.sweep import DMSweep
    C, N, P = 48, 16384, 2048
    freqs = band(C)
    dms = np.linspace(0.0, 60.0, 37)
    x = u8_data(C, N, 23)
    xd = torch.from_numpy(x).cuda()
    if dtype == "f32":
        xd = xd.float()
    sw = DMSweep(dms, freqs, DT, dtype=dtype)
    full = sw(xd)
    n_out = full.shape[1]
    xp = xd.reshape(C, N // P, P).permute(1, 0, 2).contiguous()  # [N/P][C][P]
    for x_off, cols in ((0, n_out), (3000, 5000), (n_out - 777, 777)):
        out = torch.full((len(dms), cols), -1.0, device="cuda")
        sw.sweep_pieces(xp, N, P, x_off, cols, out)
        assert torch.equal(out, full[:, x_off:x_off + cols]), (x_off, cols)
    sw.close()


@pytest.mark.parametrize("dtype", ["f32", "u8"])
def test_sweep_two_streams_interleaved(gpu, dtype):
    """One plan swept on two streams at once, with differently sized blocks
    alternating (the library's scratch is per stream and grows on demand):
    every plane equals the single-stream plane of its block."""
    import torch
    from pypulsar_amd.sweep import DMSweep
    C = 96
    freqs = band(C)
    dms = np.linspace(0.0, 300.0, 61)
    sw = DMSweep(dms, freqs, DT, dtype=dtype)
    rng = np.random.default_rng(31)
    blocks = [rng.integers(0, 256, size=(C, n), dtype=np.uint8) for n in (9000, 20000, 13000, 30000)]
    tdt = torch.uint8 if dtype == "u8" else torch.float32
    xs = [torch.from_numpy(b).cuda().to(tdt) for b in blocks]
    want = [sw(x).cpu().numpy() for x in xs]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    torch.cuda.synchronize()
    outs = []
    for rep in range(3):
        for i, x in enumerate(xs):
            st = streams[(i + rep) % 2]
            with torch.cuda.stream(st):
                outs.append((i, sw(x, stream=st)))
    torch.cuda.synchronize()
    for i, p in outs:
        np.testing.assert_array_equal(p.cpu().numpy(), want[i])
    sw.close()
