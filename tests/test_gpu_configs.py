"""GPU parity at the BASELINE.json workloads, through the product API.

* configs[0]: waterfaller-style Spectra.dedisperse(100, padval, trim=True) of a
  1024-channel 2^16-sample 8-bit filterbank in get_spectra's layout + the
  channel sum (bin/waterfaller.py:140), against the oracle;
* configs[2]: the DDplan2b two-stage executor (4096 -> 64 subbands, res
  0.5 ms: 2000 DMs, downsample 4, 40 passes x 50) at N = 2^18, sampled rows
  against oracle subband(64, subDM_k) + per-DM shifted sums;
* configs[3]: the 4096-channel x 4096-DM (0-1000) sweep at N = 2^18 against
  oracle rows, the pipelined DMShardedSweep (the bench path) against it, and
  at the full 2^22 length the size-independent properties (u8 plane == f32
  plane, rows == the independent single-DM kernel, sharded == direct);
* configs[4]: the 4096-channel 2048-DM stream of 2^18-spectrum blocks equals
  the one-shot zero-DM + downsample + sweep, bit for bit (integer zero-DM on
  the exact 16-bit path, also against oracle rows; and the float mode).

All inputs are integer-valued 8-bit data with integer pads, so every
comparison is bit-exact (float32 sums of integers < 2^24), except pad 'mean'
(1e-5 relative).
"""
import copy

import numpy as np
import pytest

from conftest import band, rel_err

DT = 64e-6
pytestmark = pytest.mark.gpu


def _u8(C, N, seed):
    return np.random.default_rng(seed).integers(0, 256, size=(C, N), dtype=np.uint8)


@pytest.mark.parametrize("pad", [0, "mean"])
def test_config0_waterfaller_dedisperse(gpu, pad):
    from oracle import spectra_oracle as orc
    from pypulsar_amd.formats.spectra import Spectra
    C, N, dm = 1024, 1 << 16, 100.0
    freqs = band(C)
    rng = np.random.default_rng(100)
    x_tc = np.clip(np.round(rng.normal(128, 16, (N, C))), 0, 255).astype(np.uint8)
    s = Spectra(freqs, DT, x_tc.T)          # filterbank.get_spectra's data.T layout
    s.dedisperse(dm, padval=pad, trim=True)
    ser = s.sum_channels().cpu().numpy()
    got = s.data
    ref, _ = orc.dedisperse(x_tc.T.astype(np.float64), freqs, DT, dm, padval=pad, trim=True)
    assert got.shape == ref.shape == (C, N - 1449)
    want_ser = orc.channel_sum(ref)
    if pad == 0:
        np.testing.assert_array_equal(got, ref)
        np.testing.assert_array_equal(ser.astype(np.float64), want_ser)
    else:
        assert rel_err(got, ref) <= 1e-5
        assert rel_err(ser, want_ser) <= 1e-5


def test_config2_two_stage_ddplan(gpu):
    import torch
    from oracle import spectra_oracle as orc
    from pypulsar_amd import delays
    from pypulsar_amd.formats.spectra import Spectra
    from pypulsar_amd.sweep import DDplanExecutor
    from pypulsar_amd.utils.ddplan import Observation
    C, N = 4096, 1 << 18
    freqs = band(C)
    plan = Observation(DT, 1400.0, 300.0, C).gen_ddplan(0.0, 1000.0, 64, 0.5)
    (step,) = plan.DDsteps
    calls = step.subband_calls()
    assert (step.downsamp, len(calls), len(calls[0][1])) == (4, 40, 50)
    x = _u8(C, N, 7)
    s = Spectra(freqs, DT, x)
    ex = DDplanExecutor(plan, freqs, DT, N, raw8=True)
    for _ in range(2):  # a second call reuses the plans and buffers
        (got_step, dms, plane) = ex(s)[0]
    plane = plane.cpu().numpy()
    ex.close()
    np.testing.assert_array_equal(dms, step.DMs)
    # oracle: downsample (channel chunks), then per sampled pass subband(64,
    # subDM_k), then per sampled DM the shifted channel sum over subbands
    dt4 = DT * 4
    xd = np.concatenate([orc.downsample(x[c:c + 512].astype(np.float64), DT, 4)[0]
                         for c in range(0, C, 512)])
    n_out = plane.shape[1]
    _, _, ctr = delays.subband_layout(freqs, 64)
    assert n_out == N // 4 - int(delays.sweep_table(step.DMs, ctr, dt4).max())
    for k in (0, 17, 39):
        subdm, cdms = calls[k]
        sub, sfreqs = orc.subband(xd, freqs, dt4, 64, subdm=subdm)
        np.testing.assert_array_equal(sfreqs, ctr)
        for j in (0, 24, 49):
            bins = orc.dedisperse_bins(cdms[j], 0.0, sfreqs, dt4)
            want = orc.shifted_sum(sub, bins)[:n_out]
            np.testing.assert_array_equal(plane[k * 50 + j].astype(np.float64), want,
                                          err_msg="pass %d DM %g" % (k, cdms[j]))
    torch.cuda.synchronize()


def test_config3_sweep_oracle_rows(gpu):
    """4096 ch x 4096 DMs (0-1000) at N = 2^18: sampled rows == oracle, and
    the pipelined DM-sharded path (one rank, 2 time batches; the bench's
    DMShardedSweep) == the direct sweep."""
    import torch
    from oracle import spectra_oracle as orc
    from pypulsar_amd.sharding import DMShardedSweep
    from pypulsar_amd.sweep import DMSweep
    C, N, D = 4096, 1 << 18, 4096
    freqs = band(C)
    dms = np.linspace(0.0, 1000.0, D)
    x = _u8(C, N, 11)
    xd = torch.from_numpy(x).cuda()
    sw = DMSweep(dms, freqs, DT, dtype="u8")
    plane = sw(xd)
    n_out = plane.shape[1]
    assert n_out == N - 14504
    table = orc.sweep_table(dms, freqs, DT)
    rows = [0, 1, 1365, 2047, 2048, 2730, 4094, 4095]
    want = orc.sweep_rows_inside(x, table[rows], n_out)
    got = plane[rows].cpu().numpy().astype(np.float64)
    np.testing.assert_array_equal(got, want)
    sw.close()
    # the bench path: time-major block, per-batch corner turn + sweep
    ds = DMShardedSweep(dms, freqs, DT, N, dtype=torch.uint8, n_batches=2, device="cuda")
    assert (ds.lo, ds.hi, ds.n_out) == (0, D, n_out)
    part = torch.from_numpy(np.ascontiguousarray(x.T)).cuda().view(2, N // 2, C)
    ds(part)
    assert torch.equal(ds.plane(), plane)
    ds.close()


@pytest.mark.parametrize("factor,g_want", [(True, 4), (2, 2)])
def test_northstar_plane(gpu, monkeypatch, factor, g_want):
    """The north-star grid (4096 ch, 2048 DMs 0-1000, DDplan2b.py:168
    arange grid spacing) at N = 2^18: the planner picks the factorised sweep
    over groups of 4 channels (and groups of 2 when asked for), its plane
    equals the channel-by-channel kernel bit for bit, and sampled rows equal
    the oracle's per-trial channel sums."""
    from pypulsar_amd import sweep as _sweep
    monkeypatch.setitem(_sweep.TEST_SWITCHES, "poison", True)  # (tests/test_gpu_factor.py)
    import torch
    from oracle import spectra_oracle as orc
    from pypulsar_amd import _lib
    from pypulsar_amd.sweep import DMSweep
    C, N, D = 4096, 1 << 18, 2048
    freqs = band(C)
    dms = np.linspace(0.0, 1000.0, D)
    x = _u8(C, N, 13)
    xd = torch.from_numpy(x).cuda()
    sw = DMSweep(dms, freqs, DT, dtype="u8", factor=factor)
    g, n_pat = sw.factor_info(_lib.U8)
    assert g == g_want and n_pat > 0, (g, n_pat)
    plane = sw(xd)
    n_out = plane.shape[1]
    assert n_out == N - 14504
    ch = DMSweep(dms, freqs, DT, dtype="u8", factor=False)
    assert ch.factor_info(_lib.U8)[0] == 0
    assert torch.equal(ch(xd), plane)
    ch.close()
    rows = [0, 1, 683, 1023, 1024, 2046, 2047]
    want = orc.sweep_rows_inside(x, orc.sweep_table(dms, freqs, DT)[rows], n_out)
    np.testing.assert_array_equal(plane[rows].cpu().numpy().astype(np.float64), want)
    sw.close()


def test_config3_timeshard_8_ranks(gpu, monkeypatch):
    """The 8-rank TIME-sharded configs[3] step (TimeShardedSweep(world=8,
    rank=r), bench.py's N > 1 default) at N = 2^18 on one GPU: each rank
    corner-turns its own input spectra (its plane columns + the max-delay
    overlap) and sweeps the whole 4096-DM grid over its columns with its own
    (factorised) plan; the 8 column blocks concatenate to the one-shot plane
    bit for bit, and sampled rows equal the oracle."""
    from pypulsar_amd import sweep as _sweep
    monkeypatch.setitem(_sweep.TEST_SWITCHES, "poison", True)  # (tests/test_gpu_factor.py)
    import torch
    from oracle import spectra_oracle as orc
    from pypulsar_amd.sharding import TimeShardedSweep
    from pypulsar_amd.sweep import DMSweep
    C, N, D, W = 4096, 1 << 18, 4096, 8
    freqs = band(C)
    dms = np.linspace(0.0, 1000.0, D)
    x = _u8(C, N, 17)
    xd = torch.from_numpy(x).cuda()
    sw = DMSweep(dms, freqs, DT, dtype="u8")
    plane = sw(xd)
    sw.close()
    block = xd.t().contiguous()                      # time-major [N, C], file order
    cols = []
    for r in range(W):
        ts = TimeShardedSweep(dms, freqs, DT, N, dtype=torch.uint8, world=W, rank=r, device="cuda")
        lo, hi = ts.input_range()
        assert hi - lo == ts.cols + 14504 and ts.a % 1024 == 0
        cols.append(ts(block[lo:hi]).clone())
        ts.close()
    got = torch.cat(cols, dim=1)
    assert got.shape == plane.shape
    assert torch.equal(got, plane)
    rows = [0, 2047, 4095]
    want = orc.sweep_rows_inside(x, orc.sweep_table(dms, freqs, DT)[rows], plane.shape[1])
    np.testing.assert_array_equal(got[rows].cpu().numpy().astype(np.float64), want)


def test_config1_full_size_f32(gpu):
    """BASELINE configs[1] at its full size -- 1024 ch x 2^20 samples x 1024
    DMs (0-1000), float32: on integer data the float32 plane equals the exact
    8-bit plane bit for bit (both factorised over groups of 2, the planner's
    choice, and the 8-bit channel-by-channel plane), and sampled rows equal
    the fused single-DM kernel (Spectra.dedispersed_series) and the oracle."""
    import torch
    from oracle import spectra_oracle as orc
    from pypulsar_amd import _lib
    from pypulsar_amd.formats.spectra import Spectra
    from pypulsar_amd.sweep import DMSweep
    C, N, D = 1024, 1 << 20, 1024
    freqs = band(C)
    dms = np.linspace(0.0, 1000.0, D)
    x = _u8(C, N, 31)
    x8 = torch.from_numpy(x).cuda()
    xf = x8.float()
    swf = DMSweep(dms, freqs, DT, dtype="f32")
    pf = swf(xf)
    assert pf.shape == (D, 1034083)
    sw8 = DMSweep(dms, freqs, DT, dtype="u8")
    assert sw8.factor_info()[0] == 2 and swf.factor_info(_lib.F32)[0] == 2
    assert torch.equal(sw8(x8), pf)
    sw8.close()
    ch = DMSweep(dms, freqs, DT, dtype="u8", factor=False)
    assert ch.factor_info()[0] == 0
    assert torch.equal(ch(x8), pf)
    ch.close()
    s = Spectra._from_device(freqs, DT, xf)
    rows = [0, 511, 1023]
    for d in rows:
        assert torch.equal(s.dedispersed_series(dms[d], padval=0, trim=True)[:pf.shape[1]], pf[d])
    want = orc.sweep_rows_inside(x, swf.table[rows], pf.shape[1])
    np.testing.assert_array_equal(pf[rows].cpu().numpy().astype(np.float64), want)
    swf.close()


def test_config1_fractional_f32_rows(gpu):
    """configs[1] grid (1024 ch, 1024 DMs 0-1000) on genuinely fractional
    float32 data (N = 2^17): sampled rows within 1e-5 relative of the
    float64 oracle -- the north_star bar at the config's full 1024-channel
    accumulation depth."""
    import torch
    from oracle import spectra_oracle as orc
    from pypulsar_amd.sweep import DMSweep
    C, N, D = 1024, 1 << 17, 1024
    freqs = band(C)
    dms = np.linspace(0.0, 1000.0, D)
    rng = np.random.default_rng(41)
    x = (rng.normal(0.0, 1.0, (C, N)) * 17.3 + 3.1).astype(np.float32)
    sw = DMSweep(dms, freqs, DT, dtype="f32")
    plane = sw(torch.from_numpy(x).cuda())
    rows = [0, 1, 300, 777, 1022, 1023]
    want = orc.sweep_rows_inside(x.astype(np.float64), sw.table[rows], plane.shape[1])
    got = plane[rows].cpu().numpy()
    for i, d in enumerate(rows):
        assert rel_err(got[i], want[i]) <= 1e-5, "row %d" % d
    sw.close()


def test_config3_rehearsal_8_ranks(gpu):
    """The 8-rank DM-sharded configs[3] step rehearsed on one GPU (VERDICT r2
    #1): rank r = DMShardedSweep(world=8, rank=r) -- its own slice of each of
    4 time batches corner-turned into the pieces block (P = N/32, a power of
    two), its work-balanced DM slice (DDplan2b.py:272-273) swept from the
    pieces at the GLOBAL trimmed width.  The 8 rank planes stacked equal the
    one-shot plane bit for bit, and sampled rows equal the oracle."""
    import torch
    from oracle import spectra_oracle as orc
    from pypulsar_amd.sharding import DMShardedSweep, split_block, trial_work
    from pypulsar_amd.sweep import DMSweep
    C, N, D, W, NB = 4096, 1 << 18, 4096, 8, 4
    freqs = band(C)
    dms = np.linspace(0.0, 1000.0, D)
    x = _u8(C, N, 21)
    block = torch.from_numpy(np.ascontiguousarray(x.T)).cuda()   # file order [N, C]
    sw = DMSweep(dms, freqs, DT, dtype="u8")
    plane = sw(block.t().contiguous())
    sw.close()
    shared, lo_prev = None, 0
    for r in range(W):
        ds = DMShardedSweep(dms, freqs, DT, N, dtype=torch.uint8, n_batches=NB,
                            work=trial_work(dms, 1), device="cuda", world=W, rank=r, x_buf=shared)
        assert ds.pieces and ds.P == N // (NB * W) and ds.lo == lo_prev
        if shared is None:
            ds.prefill(block)
            shared = ds.x
        for _ in range(2):  # a second step reuses every buffer
            ds(split_block(block, NB, W, r))
        assert torch.equal(ds.plane(), plane[ds.lo:ds.hi]), "rank %d rows differ" % r
        lo_prev = ds.hi
        ds.close()
    assert lo_prev == D
    rows = [0, 511, 512, 2047, 3584, 4095]
    want = orc.sweep_rows_inside(x, orc.sweep_table(dms, freqs, DT)[rows], plane.shape[1])
    np.testing.assert_array_equal(plane[rows].cpu().numpy().astype(np.float64), want)


def test_config3_full_length_properties(gpu):
    """4096 ch x 2^22 samples x 4096 DMs: properties that hold at any size.
    (a) the exact 8-bit (u16-image) plane equals the float32-image plane;
    (b) rows equal the independent fused single-DM kernel
        (Spectra.dedispersed_series, pdd_shift_group_sum);
    (c) a 64-DM slice swept at the GLOBAL plane width (what a DM-sharded rank
        does) equals those rows of the full plane."""
    import torch
    from pypulsar_amd.formats.spectra import Spectra
    from pypulsar_amd.sweep import DMSweep
    C, N, D = 4096, 1 << 22, 4096
    freqs = band(C)
    dms = np.linspace(0.0, 1000.0, D)
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    x8 = torch.randint(0, 256, (C, N), generator=g, device="cuda", dtype=torch.uint8)
    sw8 = DMSweep(dms, freqs, DT, dtype="u8")
    n_out = sw8.n_out(N)
    assert n_out == 4179800
    p8 = sw8(x8)
    sw8.close()
    xf = x8.float()
    chunk = 512
    for lo in range(0, D, chunk):
        swf = DMSweep(dms[lo:lo + chunk], freqs, DT, dtype="f32")
        pf = swf(xf, n_out=n_out)
        assert torch.equal(pf, p8[lo:lo + chunk]), "u8 != f32 plane in DMs [%d, %d)" % (lo, lo + chunk)
        swf.close()
        del pf
    s = Spectra._from_device(freqs, DT, xf)
    for d in (0, 1000, 2049, 4095):
        ser = s.dedispersed_series(dms[d], padval=0, trim=True)
        assert torch.equal(ser[:n_out], p8[d]), "row %d != dedispersed_series" % d
    sub = DMSweep(dms[100:164], freqs, DT, dtype="u8")
    assert sub.max_bin < N - n_out  # a low-DM slice, swept at the global width
    ps = sub(x8, n_out=n_out)
    assert torch.equal(ps, p8[100:164])
    sub.close()


@pytest.mark.parametrize("D,factor,g_want", [(2048, True, 4), (2048, 2, 2), (4096, True, 4)])
def test_northstar_full_length(gpu, monkeypatch, D, factor, g_want):
    """The north star at its full size -- 4096 ch x 2^22 samples x 2048 DMs
    (0-1000, DDplan2b.py:168 grid spacing), 8-bit -- and BASELINE configs[3]
    (the same with 4096 DMs: the default bench line's exact step) through the bench's own
    path (DMShardedSweep, one rank, 4 time batches of 2^20 spectra in file
    order, pieces layout): the planner picks groups of 4 channels (groups of
    2 when asked for: the other u16 instance at full length), the
    factorised sweep runs 4 launches (one per batch, ~1.04 M columns each)
    with its pattern image poisoned before every stage 1, and
    (a) every plane column equals the channel-by-channel kernel bit for bit
        (compared in 512-DM chunks);
    (b) sampled rows equal the independent fused single-DM kernel
        (Spectra.dedispersed_series: Spectra.dedisperse(dm, trim=True) + the
        channel sum of bin/waterfaller.py:140, formats/spectra.py:229-260)."""
    import torch
    from pypulsar_amd import _lib
    from pypulsar_amd import sweep as _sweep
    from pypulsar_amd.formats.spectra import Spectra
    from pypulsar_amd.sharding import DMShardedSweep, trial_work
    from pypulsar_amd.sweep import DMSweep
    monkeypatch.setitem(_sweep.TEST_SWITCHES, "poison", True)
    C, N, NB = 4096, 1 << 22, 4
    freqs = band(C)
    dms = np.linspace(0.0, 1000.0, D)
    g = torch.Generator(device="cuda")
    g.manual_seed(23 + D)
    x_tc = torch.randint(0, 256, (N, C), generator=g, device="cuda", dtype=torch.uint8)
    ds = DMShardedSweep(dms, freqs, DT, N, dtype=torch.uint8, n_batches=NB,
                        work=trial_work(dms, 1), device="cuda", factor=factor)
    assert ds.pieces and ds.n_out == N - 14504 == 4179800
    gg, n_pat = ds.sw.factor_info(_lib.U8)
    assert gg == g_want and n_pat > 0, (gg, n_pat)
    # delay-aligned tiles (pdd_sweep.hip fx_skew): trials skewed by up to
    # their block's delay drift at the reference group
    assert ds.sw.skew_info(_lib.U8)[0] > 64
    ds.sw.set_timing(True)
    planes = ds(x_tc.view(NB, N // NB, C))
    _, launches = ds.sw.timing_read()
    ds.sw.set_timing(False)
    assert launches == NB, launches
    edges = list(ds.col_edges)
    n_out = ds.n_out
    ds.close()
    del ds
    torch.cuda.synchronize()
    _lib.check(_lib.lib().pdd_scratch_release(), "pdd_scratch_release")
    x8 = x_tc.t().contiguous()
    del x_tc
    for lo in range(0, D, 512):
        ch = DMSweep(dms[lo:lo + 512], freqs, DT, dtype="u8", factor=False)
        assert ch.factor_info(_lib.U8)[0] == 0
        pc = ch(x8, n_out=n_out)
        for k in range(NB):
            a, b = edges[k], edges[k + 1]
            assert torch.equal(pc[:, a:b], planes[k][lo:lo + 512]), \
                "DMs [%d, %d), batch %d: factorised != channel kernel" % (lo, lo + 512, k)
        ch.close()
        del pc
    _lib.check(_lib.lib().pdd_scratch_release(), "pdd_scratch_release")
    s = Spectra._from_device(freqs, DT, x8.float())
    del x8
    for d in (0, 1, 1023, 1024, D - 2, D - 1):
        ser = s.dedispersed_series(dms[d], padval=0, trim=True)[:n_out]
        got = torch.cat([planes[k][d] for k in range(NB)])
        assert torch.equal(ser, got), "row %d != dedispersed_series" % d


def test_config2_subband_benched_size(gpu):
    """BASELINE configs[2] at the size bench.py --config subband times
    (4096 ch x 2^20 8-bit samples, DDplan2b -> 64 subbands, res 0.5 ms: 2000
    DMs at downsamp 4 in 40 passes of 50 DMs, utils/DDplan2b.py:132-168):
    sampled executor rows equal the two reference steps run on the device
    through the Spectra API -- Spectra.downsample(4) (spectra.py:329-351),
    Spectra.subband(64, subDM_k) (spectra.py:96-138) and the dedispersed
    series of the subbands at each DM of pass k (spectra.py:229-260 +
    waterfaller.py:140) -- bit for bit (integer data)."""
    import torch
    from pypulsar_amd import delays
    from pypulsar_amd.formats.spectra import Spectra
    from pypulsar_amd.sweep import DDplanExecutor
    from pypulsar_amd.utils.ddplan import Observation
    C, N = 4096, 1 << 20
    freqs = band(C)
    plan = Observation(DT, 1400.0, 300.0, C).gen_ddplan(0.0, 1000.0, 64, 0.5)
    (step,) = plan.DDsteps
    calls = step.subband_calls()
    assert (step.downsamp, len(calls), len(calls[0][1])) == (4, 40, 50)
    g = torch.Generator(device="cuda")
    g.manual_seed(29)
    x8 = torch.randint(0, 256, (C, N), generator=g, device="cuda", dtype=torch.uint8)
    ex = DDplanExecutor(plan, freqs, DT, N, raw8=True)
    s8 = Spectra(freqs, DT, x8)       # 8-bit data: the Spectra keeps its raw rows
    (got_step, dms, plane) = ex(s8)[0]
    del s8
    ex.close()
    np.testing.assert_array_equal(dms, step.DMs)
    n_out = plane.shape[1]
    _, _, ctr = delays.subband_layout(freqs, 64)
    assert n_out == N // 4 - int(delays.sweep_table(step.DMs, ctr, DT * 4).max())
    base = Spectra(freqs, DT, x8)
    base.downsample(4)
    for k in (0, 13, 26, 39):
        subdm, cdms = calls[k]
        sub = copy.deepcopy(base)
        sub.subband(64, subdm)
        np.testing.assert_array_equal(sub.freqs, ctr)
        for j in (0, 24, 49):
            ser = sub.dedispersed_series(cdms[j], padval=0, trim=True)[:n_out]
            assert torch.equal(ser, plane[k * 50 + j]), "pass %d DM %g" % (k, cdms[j])
        del sub


@pytest.mark.parametrize("zdm", ["wrap", "int", "float"])
def test_config4_stream_equals_one_shot(gpu, zdm):
    """configs[4]: 4096-ch 8-bit blocks of 2^18 spectra, zero-DM + downsample
    2 + 2048-DM sweep, streamed from pinned host memory == the one-shot
    pipeline over the whole stream.  'wrap' (the default; the reference's
    uint8 result, zero_dm_filter.py:30-39) and 'int': the exact 16-bit path
    -- the stream's sweep converts every 128 (wrap, image <= 510) / 64 (int,
    <= 1020) channels, the one-shot sweep every 64 -- also checked bit for
    bit against the oracle on a window of rows; 'float': the float32 path."""
    import torch
    from pypulsar_amd import _lib
    from pypulsar_amd._lib import call, ptr, stream_ptr
    from oracle import spectra_oracle as orc
    from pypulsar_amd.stream import StreamingSweep, prologue
    from pypulsar_amd.sweep import DMSweep
    C, D, block, ds = 4096, 2048, 1 << 18, 2
    freqs = band(C)
    dms = np.linspace(0.0, 1000.0, D)
    N = 3 * block + 100000
    x = np.random.default_rng(13).integers(0, 256, size=(N, C), dtype=np.uint8)
    st = StreamingSweep(dms, freqs, DT, block=block, downsamp=ds, zero_dm=zdm)
    assert st.ov == 7252 * ds and st.exact == (zdm != "float")
    assert st.input_max == {"wrap": 510, "int": 1020, "float": None}[zdm]
    chunks = [torch.from_numpy(x[i:i + block]).pin_memory() for i in range(0, N, block)]
    parts = [p.clone() for _, p in st(chunks)]
    st.close()
    got = torch.cat(parts, dim=1)
    xd = torch.from_numpy(x).cuda()
    if zdm != "float":
        off = 255 * ds if zdm == "int" else 0
        img = torch.empty((C, N // ds), dtype=torch.int16, device="cuda")
        prologue(xd, N, C, ds, zdm, img, off)
        sw = DMSweep(dms, freqs, DT * ds, dtype="u16")
        want = sw(img, out_bias=-float(off * C))
    else:
        f32 = torch.empty((C, N // ds), dtype=torch.float32, device="cuda")
        call("pdd_zdm_downsample", ptr(xd), _lib.U8, N, C, C, ds, 1, ptr(f32), f32.stride(0),
             stream_ptr())
        sw = DMSweep(dms, freqs, DT * ds)
        want = sw(f32)
    assert got.shape == want.shape
    assert torch.equal(got, want)
    if zdm != "float":
        # oracle window: plane columns [j0, j0 + W) need input spectra
        # [j0 ds, (j0 + W + max_bin) ds) -- across the seam of blocks 1 and 2
        W, mb = 2048, sw.max_bin
        j0 = block // ds - 1000
        win = x[j0 * ds:(j0 + W + mb) * ds]
        ref_img = orc.zdm_int_downsample(win, ds, zdm)
        rows = [0, 1, 777, 1500, 2047]
        ref = orc.sweep_rows_inside(ref_img, sw.table[rows], W)
        np.testing.assert_array_equal(got[rows, j0:j0 + W].cpu().numpy(), ref)
    sw.close()
