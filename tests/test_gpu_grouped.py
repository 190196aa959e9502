"""Grouped sweeps (pdd_sweep_*_grouped) and the two-launch DDplan executor
(execute_plan_grouped) on the GPU, against per-group DMSweeps, the per-pass
executor (Spectra.subband + per-DM sweep, i.e. the reference's per-call
semantics) and the golden two-stage plane."""
import numpy as np
import pytest

from conftest import band, rel_err, u8_data
from oracle import spectra_oracle as orc

pytestmark = pytest.mark.gpu
DT = 64e-6


def test_grouped_equals_individual(gpu):
    import torch
    from pypulsar_amd.sweep import DMSweep, GroupedSweep
    G, C, N = 5, 24, 5000
    rng = np.random.default_rng(7)
    x = torch.from_numpy(u8_data(G * C, N, 7).astype(np.float32)).cuda()
    tables, planes = [], []
    for g in range(G):
        freqs = np.sort(rng.uniform(1200, 1600, C))[::-1]
        dms = np.sort(rng.uniform(0, 40, 9))
        sw = DMSweep(dms, freqs, DT)
        tables.append(sw.table)
        planes.append(sw(x[g * C:(g + 1) * C], trim=False).cpu().numpy())
    gs = GroupedSweep(np.stack(tables))
    out = torch.full((9 * G, N), -1.0, device="cuda")
    gs(x, N, out, row_g=1, row_d=G)  # interleaved rows: trial d of group g -> d*G + g
    got = out.cpu().numpy()
    for g in range(G):
        np.testing.assert_array_equal(got[g::G], planes[g])


@pytest.mark.parametrize("dtype", ["u8", "f32"])
def test_execute_plan_grouped(gpu, golden, golden_meta, dtype):
    from pypulsar_amd.formats.spectra import Spectra
    from pypulsar_amd.sweep import execute_plan, execute_plan_grouped
    from pypulsar_amd.utils.ddplan import Observation
    C, N = 256, 1 << 15
    freqs = band(C)
    x = u8_data(C, N, 19)
    data = x if dtype == "u8" else x.astype(np.float32)
    plan = Observation(DT, 1400.0, 300.0, C).gen_ddplan(0.0, 120.0, 16, 0.5)
    assert any(st.numsub for st in plan.DDsteps)
    s = Spectra(freqs, DT, data)
    fast = execute_plan_grouped(s, plan, padval=0)
    slow = execute_plan(s, plan, padval=0, trim=True)
    for (st, dms, plane), (st2, outs) in zip(fast, slow):
        got = plane.cpu().numpy()
        ref = np.concatenate([p.cpu().numpy()[:, :got.shape[1]] for _, p in outs])
        assert got.shape[0] == len(st.DMs) and got.shape[1] <= min(p.shape[1] for _, p in outs)
        np.testing.assert_array_equal(got, ref)


def test_grouped_two_stage_golden(gpu, golden, golden_meta):
    # the reference's subband(8, 40) + dedisperse(dm, trim=True) + sum rows
    import torch
    from pypulsar_amd import delays
    from pypulsar_amd.sweep import GroupedSweep
    x = golden["sw_x"].astype(np.float32)
    freqs = golden["sw_freqs"]
    p = golden_meta["sw2"]
    nsub, C = p["nsub"], x.shape[0]
    cps = C // nsub
    t1 = delays.subband_bins(p["subDM"], freqs, DT, nsub).reshape(1, nsub, cps).transpose(1, 0, 2)
    g1 = GroupedSweep(t1)
    xd = torch.from_numpy(x).cuda()
    sub = torch.empty((nsub, x.shape[1]), device="cuda")
    g1(xd, x.shape[1], sub, row_g=1, row_d=nsub)
    _, _, ctr = delays.subband_layout(freqs, nsub)
    t2 = delays.sweep_table(golden["sw2_dms"], ctr, DT)[None]
    g2 = GroupedSweep(t2)
    want = golden["sw2_plane"]
    out = torch.empty(want.shape, device="cuda")
    g2(sub, want.shape[1], out, row_g=0, row_d=1)
    np.testing.assert_array_equal(out.cpu().numpy().astype(np.float64), want)


@pytest.mark.parametrize("factor", [1, 2, 3, 4, 8, 16, 32])
@pytest.mark.parametrize("N", [4096, 4099])
def test_downsample_u8_equals_f32(gpu, factor, N):
    """pdd_downsample_u8 (the DDplan executor's path for unmodified 8-bit
    Spectra) == pdd_downsample on the float image == the oracle, bit-exact."""
    import torch
    from pypulsar_amd._lib import call, ptr, stream_ptr
    C = 37
    x = u8_data(C, N, factor)
    xu = torch.from_numpy(x).cuda()
    xf = xu.float()
    n = N // factor
    a = torch.zeros((C, n), device="cuda")
    b = torch.zeros((C, n), device="cuda")
    call("pdd_downsample_u8", ptr(xu), C, N, N, factor, ptr(a), n, stream_ptr())
    call("pdd_downsample", ptr(xf), C, N, N, factor, ptr(b), n, stream_ptr())
    want, _ = orc.downsample(x.astype(np.float64), DT, factor)
    np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy())
    np.testing.assert_array_equal(a.cpu().numpy().astype(np.float64), want)


@pytest.mark.parametrize("padval", [0, 7, 3.5, "mean"])
def test_executor_u16_steps_and_pads(gpu, padval):
    """DDplanExecutor on 8-bit rows: downsample <= 4 steps run on the exact
    16-bit path (pdd_downsample_u8_u16 + u16 grouped sweep) for integer pads
    and fall back to the float32 image otherwise; ds 8 steps are float32.
    Every plane equals the per-pass executor (Spectra.subband + dedisperse),
    bit for bit for integer pads, 1e-5 for fractional ones."""
    from pypulsar_amd.formats.spectra import Spectra
    from pypulsar_amd.sweep import DDplanExecutor, execute_plan
    from pypulsar_amd.utils.ddplan import Observation
    C, N = 256, 1 << 15
    freqs = band(C)
    x = u8_data(C, N, 23)
    plan = Observation(DT, 1400.0, 300.0, C).gen_ddplan(0.0, 400.0, 16, 0.5)
    assert [st.downsamp for st in plan.DDsteps] == [4, 8]
    s = Spectra(freqs, DT, x)
    ex = DDplanExecutor(plan, freqs, DT, N, raw8=True)
    assert [st.u16 for st in ex.steps] == [True, False]
    fast = ex(s, padval=padval)
    slow = execute_plan(s, plan, padval=padval, trim=True)
    for (st, dms, plane), (st2, outs) in zip(fast, slow):
        got = plane.cpu().numpy()
        ref = np.concatenate([p.cpu().numpy()[:, :got.shape[1]] for _, p in outs])
        if isinstance(padval, str) or not float(padval).is_integer():
            assert rel_err(got, ref) <= 1e-5
        else:
            np.testing.assert_array_equal(got, ref)
    ex.close()


@pytest.mark.parametrize("ds", [2, 3, 4])
@pytest.mark.parametrize("padval", [0, 17, "rotate"])
@pytest.mark.parametrize("layout", ["vec16", "vec", "bytes"])
def test_sweep_ds_fused_downsample(gpu, ds, padval, layout):
    """pdd_sweep_execute_ds (8-bit rows co-added by ds inside the 16-bit
    interleave pre-pass) == the oracle's Spectra.downsample + sweep, bit for
    bit, on a ragged raw length, over the full width (pads/rotation at the
    edges).  Row layouts: 16-B aligned rows (the 16-byte-load kernel), rows
    aligned to ds only, and unaligned rows (byte loads).  Grouped plans too."""
    import torch
    from pypulsar_amd.sweep import DMSweep, GroupedSweep
    C, n_raw = 96, (1 << 13) + 3
    width = {"vec16": 8208, "vec": 8212, "bytes": 8208}[layout]
    x = u8_data(C, width, 40 + ds)
    xt = torch.from_numpy(x).cuda()
    o = 1 if layout == "bytes" else 0
    x8 = xt[:, o:o + n_raw]
    ref8 = x[:, o:o + n_raw]
    freqs = band(C)
    dms = np.linspace(0.0, 60.0, 37)
    sw = DMSweep(dms, freqs, DT * ds, dtype="u16")
    N = n_raw // ds
    got = sw.sweep_ds(x8, ds, padval=padval, n_out=N).cpu().numpy()
    xd, _ = orc.downsample(ref8.astype(np.float64), DT, ds)
    ref = orc.sweep_plane(xd, sw.table, padval=padval, n_out=N)
    np.testing.assert_array_equal(got, ref)
    # grouped: two groups of C/2 channels, rows interleaved
    t2 = np.stack([sw.table[:, :C // 2], sw.table[:, C // 2:]])
    gs = GroupedSweep(t2, "u16")
    out = torch.full((2 * len(dms), N), -1.0, device="cuda")
    mode = 1 if isinstance(padval, str) else 0
    pv = None if mode else torch.full((C,), float(padval), device="cuda")
    from pypulsar_amd import _lib
    gs.execute_ds(x8, ds, N, out, row_g=1, row_d=2,
                  pad_mode=_lib.PAD_ROTATE if mode else _lib.PAD_VALUE, padvals=pv)
    g = out.cpu().numpy()
    for k in range(2):
        refk = orc.sweep_plane(xd[k * C // 2:(k + 1) * C // 2], t2[k], padval=padval, n_out=N)
        np.testing.assert_array_equal(g[k::2], refk)
    sw.close()
    gs.close()


@pytest.mark.parametrize("ds", [2, 3, 4])
@pytest.mark.parametrize("padval", [0, 17, "rotate"])
@pytest.mark.parametrize("factor", ["force4", "force2", True])
def test_sweep_ds_factorised(gpu, ds, padval, factor, monkeypatch):
    """sweep_ds (and so DDplanExecutor's one-stage steps at downsamp 2..4) on
    a dtype='u16' plan that IS factorised: the interleave pre-pass co-adds
    the raw rows, stage 1 builds the patterns from that image, and the plane
    equals the oracle's Spectra.downsample + per-trial sweep bit for bit.
    factor=True: whatever the planner picks for this grid."""
    from pypulsar_amd import sweep as _sweep
    monkeypatch.setitem(_sweep.TEST_SWITCHES, "poison", True)  # (tests/test_gpu_factor.py)
    import torch
    from pypulsar_amd import _lib
    from pypulsar_amd.sweep import DMSweep
    C, n_raw = 128, (1 << 14) + 5
    x = u8_data(C, n_raw, 60 + ds)
    x8 = torch.from_numpy(x).cuda()
    dms = np.linspace(0.0, 12.0, 96)
    sw = DMSweep(dms, band(C), DT * ds, dtype="u16", factor=factor)
    g = sw.factor_info(_lib.U16)[0]
    if factor is not True:
        assert g == int(factor[-1]), g
    N = n_raw // ds
    got = sw.sweep_ds(x8, ds, padval=padval, n_out=N).cpu().numpy()
    xd, _ = orc.downsample(x.astype(np.float64), DT, ds)
    ref = orc.sweep_plane(xd, sw.table, padval=padval, n_out=N)
    np.testing.assert_array_equal(got, ref)
    sw.close()


@pytest.mark.parametrize("ds", [1, 2, 4])
@pytest.mark.parametrize("padval", [0, 9])
def test_subband_chain_equals_stages(gpu, ds, padval):
    """pdd_subband_chain (stage 1 writes stage 2's float32 quarters image
    directly) == stage 1 into a subband plane + stage 2 over it, bit for bit,
    on a ragged block; and one row against the oracle's Spectra.subband +
    dedisperse + channel sum.  ds 1: 8-bit stage 1; ds 2/4: co-added on the
    fly (16-bit stage 1)."""
    import torch
    from pypulsar_amd import _lib, delays
    from pypulsar_amd._lib import ptr
    from pypulsar_amd.sweep import GroupedSweep
    C, nsub, n_raw = 128, 8, (1 << 14) + 5 * ds
    cps = C // nsub
    freqs = band(C)
    dt = DT * ds
    x = u8_data(C, n_raw + 11, 70 + ds)[:, :n_raw].copy()
    x8 = torch.from_numpy(x).cuda()
    subdms = [5.0, 15.0, 25.0]
    dms = [np.linspace(sd - 5, sd + 5, 6, endpoint=False) for sd in subdms]
    t1 = np.stack([delays.subband_bins(sd, freqs, dt, nsub) for sd in subdms])
    t1 = t1.reshape(len(subdms), nsub, cps).transpose(1, 0, 2)
    g1 = GroupedSweep(t1, "u8" if ds == 1 else "u16")
    _, _, ctr = delays.subband_layout(freqs, nsub)
    t2 = np.stack([delays.sweep_table(d, ctr, dt) for d in dms])
    g2 = GroupedSweep(t2, "f32")
    N = n_raw // ds
    n_out = N - int(t2.max())
    pv1 = torch.full((C,), float(padval), device="cuda")
    pv2 = torch.full((len(subdms) * nsub,), float(padval), device="cuda")
    # stages apart
    sub = torch.empty((len(subdms) * nsub, N), device="cuda")
    if ds == 1:
        g1(x8, N, sub, row_g=1, row_d=nsub, pad_mode=_lib.PAD_VALUE, padvals=pv1)
    else:
        g1.execute_ds(x8, ds, N, sub, row_g=1, row_d=nsub, pad_mode=_lib.PAD_VALUE, padvals=pv1)
    ref = torch.full((len(subdms) * 6, n_out), -1.0, device="cuda")
    g2(sub, n_out, ref, row_g=6, row_d=1, pad_mode=_lib.PAD_VALUE, padvals=pv2)
    got = torch.full_like(ref, -2.0)
    _lib.call("pdd_subband_chain", g1._plan, ptr(x8), n_raw, x8.stride(0), ds, _lib.PAD_VALUE,
              ptr(pv1), g2._plan, ptr(pv2), ptr(got), got.stride(0), n_out, 6, 1,
              _lib.stream_ptr())
    got = got.cpu().numpy()
    np.testing.assert_array_equal(got, ref.cpu().numpy())
    # oracle: pass 1, DM 2 -> Spectra.downsample + subband + dedisperse + sum
    xd, _ = orc.downsample(x.astype(np.float64), DT, ds)
    subd, sfreqs = orc.subband(xd, freqs, dt, nsub, subdm=subdms[1], padval=padval)
    ded, _ = orc.dedisperse(subd, sfreqs, dt, dms[1][2], cur_dm=0.0, padval=padval)
    want = orc.channel_sum(ded)
    np.testing.assert_array_equal(got[6 + 2], want[:n_out])
    g1.close()
    g2.close()


@pytest.mark.parametrize("case", ["u8_const255", "u16_const1023", "u8_extremes"])
def test_grouped_short_tiling_saturated(gpu, case):
    """Grouped short grids (40 trials per group) take the 8-wave DB-40 tiling
    (variant 100: 8 trials per compute wave, byte-wide carry counts) up to the
    plan's bound C x input <= 255 * 2^15.  const: every plane value equals
    C x v; extremes (random 0 / 255): each group's rows equal the
    single-group DMSweep over its channels (the 48-trial tiling, u16 carry
    words).  Above the bound the plan falls back to the 48-trial tiling."""
    import torch
    from pypulsar_amd import _lib
    from pypulsar_amd.sweep import DMSweep, GroupedSweep
    N, D, G = 4096, 40, 2
    if case == "u16_const1023":
        C, dtype, v = 8167, "u16", 1023
    else:
        C, dtype, v = 32768, "u8", 255
    freqs = band(C)
    dms = np.linspace(0.0, 2.0, D)
    sw = DMSweep(dms, freqs, DT, dtype=dtype, factor=False)
    gs = GroupedSweep(np.stack([sw.table] * G), dtype)
    assert gs.info()["variant"] == 100, gs.info()
    if case == "u8_extremes":
        g = torch.Generator(device="cuda")
        g.manual_seed(11)
        x = torch.randint(0, 2, (G * C, N), generator=g, device="cuda", dtype=torch.uint8) * 255
    else:
        x = torch.full((G * C, N), v, device="cuda",
                       dtype=torch.uint8 if dtype == "u8" else torch.int16)
    n_out = sw.n_out(N, True)
    out = torch.full((G * D, n_out), -1.0, device="cuda")
    pv = torch.full((G * C,), float(v), device="cuda")
    gs(x, n_out, out, row_g=1, row_d=G, pad_mode=_lib.PAD_VALUE, padvals=pv)
    if case == "u8_extremes":
        for k in range(G):
            want = sw(x[k * C:(k + 1) * C])
            assert torch.equal(out[k::G], want), k
    else:
        assert 255 * 32768 - 1023 <= v * C <= 255 * 32768
        assert torch.all(out == float(v * C)), (out.min().item(), out.max().item())
    # one channel more than the bound: not the byte-carry tiling
    big = GroupedSweep(np.stack([np.concatenate([sw.table, sw.table[:, :1]], 1)] * G)
                       if v * (C + 1) > 255 * 32768 else np.stack([sw.table] * G), dtype)
    if v * (C + 1) > 255 * 32768:
        assert big.info()["variant"] != 100, big.info()
    big.close()
    gs.close()
    sw.close()
