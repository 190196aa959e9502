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
