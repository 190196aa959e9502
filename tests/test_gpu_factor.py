"""Exact factorised 8-bit sweep (pdd_sweep.hip k_fx_patterns + k_sweep_il
FX): each group of 4 adjacent channels is summed once per distinct
relative-shift pattern, and every trial adds its pattern series at the
group's base shift -- the same integer samples as the channel-by-channel sum
(formats/spectra.py:229-260 dedisperse + bin/waterfaller.py:140 channel sum,
per trial), so the planes must be BIT-IDENTICAL to the oracle's and to the
channel-by-channel kernel's."""
import numpy as np
import pytest

from conftest import band, u8_data
from oracle import spectra_oracle as orc

DT = 64e-6


@pytest.fixture(autouse=True)
def poison_patterns(monkeypatch):
    """Every factorised sweep here first fills its pattern image with 0xFF
    bytes (pdd_sweep_plan_set_poison): stage 1 writes only the row elements each
    pattern's trials read (fx_build's per-pattern ranges), so a sum reading
    an unwritten element turns into a NaN / an overflowed lane, not a stale
    value that happens to match."""
    from pypulsar_amd import sweep
    monkeypatch.setitem(sweep.TEST_SWITCHES, "poison", True)


@pytest.mark.gpu
@pytest.mark.parametrize("pad", [0, 7, "rotate"])
@pytest.mark.parametrize("descending", [True, False])
@pytest.mark.parametrize("C,g", [(32, 4), (36, 4), (36, 2), (34, 2)])
def test_factor_small_grids_vs_oracle(gpu, pad, descending, C, g):
    """Forced factorisation on small grids, groups of 4 and of 2 channels:
    pads (value / rotate) past the block edge (trim=False), ascending bands
    (negative relative shifts), odd group counts (C = 36 in 4s: 9 groups; C =
    34 in 2s: 17 groups -- the last pair ends in a zero group)."""
    import torch
    from pypulsar_amd.sweep import DMSweep
    N, D = 6000, 64
    freqs = band(C, descending=descending)
    x = u8_data(C, N, 31 + C)
    # (a grid whose group pairs' pattern windows fit one chunk buffer: with
    # 9-MHz channels every trial of a wider grid has its own pattern)
    dms = np.linspace(0, 3.0 if C == 32 else 4.0, D)
    sw = DMSweep(dms, freqs, DT, dtype="u8", factor="force" if g == 4 else "force2")
    assert sw.factor_info()[0] == g
    for trim in (True, False):
        plane = sw(torch.from_numpy(x).cuda(), padval=pad, trim=trim).cpu().numpy()
        tab = orc.sweep_table(dms, freqs, DT)
        n_out = plane.shape[1]
        want = orc.sweep_plane(x.astype(np.float64), tab, pad, n_out=n_out)
        np.testing.assert_array_equal(plane.astype(np.float64), want,
                                      err_msg="pad %r trim %s" % (pad, trim))
    sw.close()


@pytest.mark.gpu
def test_factor_config1_geometry_equals_channel_sweep(gpu):
    """BASELINE configs[1] geometry (1024 ch x 1024 DM, 0-1000 pc/cc) on 8-bit
    data at N = 2^17: the planner factorises over groups of 2 (7944 patterns;
    groups of 4, 25k patterns for 256 groups, only when forced), and both
    planes equal the channel-by-channel kernel's bit for bit, and the
    oracle's rows."""
    import torch
    from pypulsar_amd.sweep import DMSweep
    C, N, D = 1024, 1 << 17, 1024
    freqs = band(C)
    dms = np.linspace(0, 1000, D)
    x = u8_data(C, N, 41)
    xd = torch.from_numpy(x).cuda()
    auto = DMSweep(dms, freqs, DT, dtype="u8")
    assert auto.factor_info()[0] == 2
    fx = DMSweep(dms, freqs, DT, dtype="u8", factor="force")
    g, n_pat = fx.factor_info()
    assert g == 4 and 0 < n_pat < 32 * C
    plain = DMSweep(dms, freqs, DT, dtype="u8", factor=False)
    assert plain.factor_info()[0] == 0
    a = fx(xd)
    b = plain(xd)
    assert torch.equal(a, b)
    assert torch.equal(auto(xd), b)
    tab = orc.sweep_table(dms, freqs, DT)
    rows = [0, 1, 511, 777, 1023]
    want = orc.sweep_plane(x.astype(np.float64), tab[rows], 0, n_out=a.shape[1])
    np.testing.assert_array_equal(a[rows].cpu().numpy().astype(np.float64), want)
    fx.close()
    plain.close()
    auto.close()


@pytest.mark.gpu
def test_factor_segments_and_column_offsets(gpu, monkeypatch):
    """A segment budget that splits the factorised sweep into several
    launches (each with its own interleave + pattern image), and a column
    range [x_off, x_off + n_out) swept from the pieces layout (the DM-sharded
    path): both equal the one-shot channel-by-channel plane."""
    import torch
    from pypulsar_amd.sweep import DMSweep
    C, N, D = 1024, 1 << 16, 512
    freqs = band(C)
    dms = np.linspace(0, 500, D)
    x = u8_data(C, N, 43)
    xd = torch.from_numpy(x).cuda()
    plain = DMSweep(dms, freqs, DT, dtype="u8", factor=False)
    ref = plain(xd)
    fx = DMSweep(dms, freqs, DT, dtype="u8", factor="force")
    g, n_pat = fx.factor_info()
    assert g == 4
    # image rows (channels + patterns + zero rows) x (delay span + ~3000
    # elements of eighths): three or four segments of N
    rows = C + 1 + n_pat + 1
    fx.set_segment_bytes(rows * 16 * (fx.max_bin + 64 + 3000))
    seg = fx(xd)
    fx.set_segment_bytes(0)
    assert torch.equal(seg, ref)
    # pieces layout [N/P][C][P] and a column window
    P = 1 << 13
    xp = xd.view(C, N // P, P).permute(1, 0, 2).contiguous()
    x_off, n_cols = 3000, 20000
    out = torch.empty((D, n_cols), dtype=torch.float32, device="cuda")
    fx.sweep_pieces(xp, N, P, x_off, n_cols, out)
    assert torch.equal(out, ref[:, x_off:x_off + n_cols])
    fx.close()
    plain.close()


@pytest.mark.gpu
def test_factor_chosen_for_config3_grid(gpu):
    """BASELINE configs[3] grid (4096 ch x 4096 DMs, 0-1000 pc/cc): the
    planner's cost model takes the factorised sweep."""
    from pypulsar_amd.sweep import DMSweep
    sw = DMSweep(np.linspace(0, 1000, 4096), band(4096), DT, dtype="u8")
    g, n_pat = sw.factor_info()
    assert g == 4 and n_pat > 1024
    sw.close()
    # the north star's grid (2048 DMs): groups of 4 as well (measured, round
    # 5: stage 2 69.0 ms per launch against 81.2 with groups of 2)
    sw = DMSweep(np.linspace(0, 1000, 2048), band(4096), DT, dtype="u8")
    assert sw.factor_info()[0] == 4
    sw.close()


@pytest.mark.gpu
@pytest.mark.parametrize("input_max", [None, 510])
def test_factor_16bit_input_vs_oracle(gpu, input_max):
    """16-bit input (samples <= 1023: the offset zero-DM + downsample image of
    the stream; <= 510 for its uint8-wrap mode, input_max) factorised in
    groups of 4 and of 2: pattern sums <= 4 x 1023 stay exact in the packed
    u16 lanes, which flush every floor(65535 / (g x max)) groups."""
    import torch
    from pypulsar_amd.sweep import DMSweep
    C, N, D = 36, 6000, 64
    freqs = band(C)
    vmax = 1023 if input_max is None else input_max
    rng = np.random.default_rng(7)
    x = rng.integers(0, vmax + 1, size=(C, N)).astype(np.int16)
    dms = np.linspace(0, 4.0, D)
    tab = orc.sweep_table(dms, freqs, DT)
    want = orc.sweep_plane(x.astype(np.float64), tab, 0)
    for mode, g in (("force4", 4), ("force2", 2)):
        sw = DMSweep(dms, freqs, DT, dtype="u16", input_max=input_max, factor=mode)
        assert sw.factor_info(2)[0] == g
        plane = sw(torch.from_numpy(x).cuda()).cpu().numpy().astype(np.float64)
        np.testing.assert_array_equal(plane, want, err_msg="g %d" % g)
        sw.close()


@pytest.mark.gpu
@pytest.mark.parametrize("pad", [0, 3.5, "mean", "rotate"])
@pytest.mark.parametrize("descending", [True, False])
@pytest.mark.parametrize("C,g", [(36, 4), (34, 2)])
def test_factor_f32_small_grids_vs_oracle(gpu, pad, descending, C, g):
    """Factorised FLOAT32 sweeps (k_fx_patterns_xf + k_sweep_il<..., FX> on the
    float32 quarters): forced groups of 4 / 2, value / statistical / rotate
    pads past the block edge, both band orders.  Integer-valued data with an
    integer pad are bit-exact (every partial sum is an integer < 2^24);
    fractional data and fractional pads within the float32 bar (1e-5 of the
    row's max)."""
    import torch
    from conftest import rel_err
    from pypulsar_amd.sweep import DMSweep
    N, D = 6000, 64
    freqs = band(C, descending=descending)
    # (DB = 56 trials per block: a narrower grid than the u16 tests' for
    # groups of 4, whose pairs' pattern windows must fit one chunk buffer)
    dms = np.linspace(0, 3.0 if g == 4 else 4.0, D)
    tab = orc.sweep_table(dms, freqs, DT)
    sw = DMSweep(dms, freqs, DT, dtype="f32", factor="force4" if g == 4 else "force2")
    assert sw.factor_info(0)[0] == g
    xi = u8_data(C, N, 51 + C).astype(np.float32)
    xf = np.random.default_rng(52 + C).normal(3.0, 1.5, (C, N)).astype(np.float32)
    for data, exact in ((xi, pad in (0, "rotate")), (xf, False)):
        for trim in (True, False):
            plane = sw(torch.from_numpy(data).cuda(), padval=pad, trim=trim).cpu().numpy()
            want = orc.sweep_plane(data.astype(np.float64), tab, pad, n_out=plane.shape[1])
            if exact:
                np.testing.assert_array_equal(plane.astype(np.float64), want)
            else:
                assert rel_err(plane, want) <= 1e-5, (pad, trim, rel_err(plane, want))
    sw.close()


@pytest.mark.gpu
def test_factor_f32_config1_geometry(gpu):
    """BASELINE configs[1] geometry (1024 ch x 1024 DM, 0-1000 pc/cc, float32)
    at N = 2^17, factorised over groups of 2 (forced): integer-valued data
    equal the channel-by-channel f32 kernel bit for bit, fractional data the
    oracle rows within 1e-5."""
    import torch
    from conftest import rel_err
    from pypulsar_amd.sweep import DMSweep
    C, N, D = 1024, 1 << 17, 1024
    freqs = band(C)
    dms = np.linspace(0, 1000, D)
    fx = DMSweep(dms, freqs, DT, dtype="f32", factor="force2")
    assert fx.factor_info(0)[0] == 2
    plain = DMSweep(dms, freqs, DT, dtype="f32", factor=False)
    xi = torch.from_numpy(u8_data(C, N, 43).astype(np.float32)).cuda()
    assert torch.equal(fx(xi), plain(xi))
    xf = np.random.default_rng(44).normal(0.0, 1.0, (C, N)).astype(np.float32)
    a = fx(torch.from_numpy(xf).cuda())
    rows = [0, 1, 511, 1023]
    want = orc.sweep_plane(xf.astype(np.float64), orc.sweep_table(dms, freqs, DT)[rows], 0,
                           n_out=a.shape[1])
    assert rel_err(a[rows].cpu().numpy(), want) <= 1e-5
    fx.close()
    plain.close()


@pytest.mark.gpu
@pytest.mark.parametrize("pad", [0, 7, "rotate"])
@pytest.mark.parametrize("descending", [True, False])
@pytest.mark.parametrize("mode", ["force4", "force2"])
def test_factor_delay_aligned_tiles(gpu, pad, descending, mode):
    """Delay-aligned factorised tiles (pdd_sweep.hip fx_skew): each trial's
    time tile is skewed by its delay at a mid-band reference group, here by up
    to ~175 samples (two extra time tiles per segment), so tiles of one trial
    block store different column ranges and the first / last tiles store only
    part of their elements.  The plane equals the plane-aligned tiles' plane
    and the oracle's bit for bit: value / rotate pads, trim on and off, both
    band orders, a grid over two trial blocks with a partial second block."""
    import torch
    from pypulsar_amd.sweep import DMSweep
    C, N, D = 256, 6000, 200
    freqs = band(C, descending=descending)
    x = u8_data(C, N, 61)
    xd = torch.from_numpy(x).cuda()
    dms = np.linspace(0, 60.0, D)
    sk = DMSweep(dms, freqs, DT, dtype="u8", factor=mode)
    al = DMSweep(dms, freqs, DT, dtype="u8", factor=mode, skew=False)
    assert sk.factor_info()[0] == al.factor_info()[0] == int(mode[-1])
    s_max, extra = sk.skew_info()
    assert s_max > 128 and extra >= 2, (s_max, extra)
    assert al.skew_info() == (0, 0)
    tab = orc.sweep_table(dms, freqs, DT)
    for trim in (True, False):
        a = sk(xd, padval=pad, trim=trim)
        b = al(xd, padval=pad, trim=trim)
        assert torch.equal(a, b), (pad, trim)
        want = orc.sweep_plane(x.astype(np.float64), tab, pad, n_out=a.shape[1])
        np.testing.assert_array_equal(a.cpu().numpy().astype(np.float64), want,
                                      err_msg="pad %r trim %s" % (pad, trim))
    sk.close()
    al.close()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["u8_const255", "u16_const1023", "u8_extremes"])
def test_factor_saturated_accumulators(gpu, case):
    """The packed-u16 accumulation at its limits (k_sweep_il normalise16 /
    HI8 carry bytes): plane sums up to 255 * 2^15 (the plan's HI8 bound,
    C * input bound <= 255 * 32768), lanes flushed every floor(32767 / (g x
    bound)) groups.
      u8_const255: 32 768 channels of 255 -- every sum 255 * C = 8 355 840, the
        carry bytes at 255;
      u16_const1023: 8164 channels of 1023 (groups of 4: flush every 8
        groups, = the chunk's group count) -- sums 8 351 772;
      u8_extremes: random 0 / 255 samples on 32 768 channels -- the factorised
        plane equals the channel-by-channel kernel's (u16 carries, DB 72)."""
    import torch
    from pypulsar_amd import _lib
    from pypulsar_amd.sweep import DMSweep
    N, D = 4096, 96
    if case == "u16_const1023":
        C, dtype, code, v = 8164, "u16", _lib.U16, 1023
    else:
        C, dtype, code, v = 32768, "u8", _lib.U8, 255
    freqs = band(C)
    dms = np.linspace(0.0, 2.0, D)
    if case == "u8_extremes":
        g = torch.Generator(device="cuda")
        g.manual_seed(9)
        x = (torch.randint(0, 2, (C, N), generator=g, device="cuda", dtype=torch.uint8) * 255)
    elif dtype == "u8":
        x = torch.full((C, N), v, dtype=torch.uint8, device="cuda")
    else:
        x = torch.full((C, N), v, dtype=torch.int16, device="cuda")
    sw = DMSweep(dms, freqs, DT, dtype=dtype, factor="force4")
    assert sw.factor_info(code)[0] == 4
    plane = sw(x)
    assert plane.shape[1] > 2048
    if case == "u8_extremes":
        ch = DMSweep(dms, freqs, DT, dtype=dtype, factor=False)
        assert ch.factor_info(code)[0] == 0
        assert torch.equal(plane, ch(x))
        ch.close()
    else:
        assert 255 * 32768 - 4 * 1023 <= v * C <= 255 * 32768
        assert torch.all(plane == float(v * C)), (plane.min().item(), plane.max().item())
    sw.close()


@pytest.mark.gpu
def test_factor_staged_execution_on_cu_partitioned_streams(gpu):
    """pdd_sweep_execute_stage: stage 1 of block k+1 into one pattern buffer
    on a stream of 32 CUs while stage 2 of block k reads the other buffer on
    a stream of the remaining CUs (pdd_stream_create_cu_mask): every plane
    equals the one-shot factorised sweep (stage 3) and the channel kernel."""
    import torch
    from pypulsar_amd.sweep import DMSweep, cu_masked_stream, cu_stream_release
    C, N, D = 1024, 1 << 16, 512
    freqs = band(C)
    dms = np.linspace(0, 500, D)
    sw = DMSweep(dms, freqs, DT, dtype="u8", factor="force")
    assert sw.factor_info()[0] == 4
    plain = DMSweep(dms, freqs, DT, dtype="u8", factor=False)
    n_out = sw.n_out(N)
    xs = [torch.from_numpy(u8_data(C, N, 70 + k)).cuda() for k in range(3)]
    refs = [plain(x) for x in xs]
    nb = sw.pattern_bytes(n_out)
    assert nb > 0 and plain.pattern_bytes(n_out) == 0
    bufs = [torch.empty(nb, dtype=torch.uint8, device="cuda") for _ in range(2)]
    outs = [torch.full((D, n_out), -1.0, device="cuda") for _ in range(3)]
    s1 = cu_masked_stream(range(224, 256))
    s2 = cu_masked_stream(range(224))
    done1 = [torch.cuda.Event() for _ in range(3)]
    done2 = [torch.cuda.Event() for _ in range(3)]
    torch.cuda.synchronize()
    for k in range(3):
        if k >= 2:
            s1.wait_event(done2[k - 2])  # buffer k % 2 is free once stage 2 of k - 2 ran
        sw.sweep_pieces_stage(xs[k], N, 0, 0, n_out, None, bufs[k % 2], 1, stream=s1)
        done1[k].record(s1)
        s2.wait_event(done1[k])
        sw.sweep_pieces_stage(xs[k], N, 0, 0, n_out, outs[k], bufs[k % 2], 2, stream=s2)
        done2[k].record(s2)
    torch.cuda.synchronize()
    for k in range(3):
        assert torch.equal(outs[k], refs[k]), k
    one = torch.empty_like(outs[0])
    sw.sweep_pieces_stage(xs[0], N, 0, 0, n_out, one, bufs[0], 3)
    assert torch.equal(one, refs[0])
    with pytest.raises(Exception):
        sw.sweep_pieces_stage(xs[0], N, 0, 0, n_out, one, bufs[0][: nb // 2], 2)
    cu_stream_release(s1)
    cu_stream_release(s2)
    sw.close()
    plain.close()
