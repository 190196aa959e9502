"""Host-side product logic (CPU only): bit-exact delay tables and the DDplan
grid generator against the reference's golden fixtures."""
import numpy as np
import pytest

from pypulsar_amd import delays
from pypulsar_amd.utils import ddplan
from conftest import GOLDEN, band
import os

DT = 64e-6


@pytest.mark.parametrize("C", [64, 1024, 4096])
@pytest.mark.parametrize("tag", ["desc", "asc"])
def test_dedisperse_bins_bit_exact(golden, C, tag):
    key = "bins_C%d_%s" % (C, tag)
    freqs = golden[key + "_freqs"]
    assert np.array_equal(freqs, band(C, tag == "desc"))
    for i, dm in enumerate(golden["bins_dms"]):
        assert np.array_equal(delays.dedisperse_bins(dm, freqs, DT), golden[key][i])
    # the vectorised [D, C] table must be bit-identical row by row
    tab = delays.sweep_table(golden["bins_dms"], freqs, DT)
    assert np.array_equal(tab, golden[key])


def test_sweep_table_grid(golden):
    tab = delays.sweep_table(golden["bins_grid_dms"], band(1024), DT)
    assert np.array_equal(tab, golden["bins_grid"])


def test_sweep_table_cur_dm():
    freqs = band(256)
    for cur in (0.0, 37.5, 100.0):
        for dm in (0.0, 12.5, 50.0, 333.0):
            row = delays.sweep_table([dm], freqs, DT, cur_dm=cur)[0]
            assert np.array_equal(row, delays.dedisperse_bins(dm, freqs, DT, cur_dm=cur))


@pytest.mark.parametrize("tag", ["desc", "asc"])
@pytest.mark.parametrize("nsub", [8, 32])
def test_subband_bins(golden, golden_meta, tag, nsub):
    freqs = golden["sb_freqs_" + tag]
    for si, subdm in enumerate(golden_meta["subdms"]):
        if subdm is None:
            continue
        k = "sb_%s_n%d_s%d_p0" % (tag, nsub, si)
        assert np.array_equal(delays.subband_bins(subdm, freqs, DT, nsub), golden[k + "_bins"])
        _, _, ctr = delays.subband_layout(freqs, nsub)
        assert np.array_equal(ctr, golden[k + "_freqs"])


def test_known_answer_delay():
    # k_DM = 1/0.000241 s MHz^2 / (pc cm^-3): DM 100 at 1000 MHz -> 0.41494 s
    assert delays.delay_from_DM(100.0, 1000.0) == pytest.approx(100.0 / 241.0, rel=1e-15)
    assert delays.delay_from_DM(100.0, np.array([0.0, -5.0]))[0] == 0.0
    # guess_DMstep o dm_smear = identity (DDplan2b.py:447)
    for dt_, bw, f in [(64e-6, 300.0, 1400.0), (1e-3, 10.0, 350.0)]:
        dm = delays.guess_DMstep(dt_, bw, f)
        assert delays.dm_smear(dm, bw, f) == pytest.approx(dt_, rel=1e-12)


def test_int32_guard():
    with pytest.raises(OverflowError):
        delays.to_int32(np.array([2 ** 31]))


@pytest.mark.parametrize("i", range(6))
def test_ddplan_matches_reference(golden, golden_meta, i):
    meta = golden_meta["ddplans"][i]
    p = meta["params"]
    obs = ddplan.Observation(p["dt"], p["fctr"], p["BW"], p["numchan"], p["numsamp"])
    plan = obs.gen_ddplan(p["lo"], p["hi"], p["nsub"], p["res"])
    assert len(plan.DDsteps) == len(meta["steps"])
    for j, (st, ref) in enumerate(zip(plan.DDsteps, meta["steps"])):
        assert st.loDM == ref["loDM"] and st.hiDM == ref["hiDM"] and st.dDM == ref["dDM"]
        assert st.downsamp == ref["downsamp"] and st.numDMs == ref["numDMs"]
        assert st.dsubDM == ref["dsubDM"] and st.numprepsub == ref["numprepsub"]
        if p["nsub"]:
            assert st.DMs_per_prepsub == ref["DMs_per_prepsub"]
        assert st.BW_smearing == ref["BW_smearing"] and st.sub_smearing == ref["sub_smearing"]
        assert np.array_equal(st.DMs, golden["ddplan%d_step%d_DMs" % (i, j)])
        assert np.array_equal(st.tot_smear, golden["ddplan%d_step%d_totsmear" % (i, j)])
    assert np.array_equal(plan.work_fracts, golden["ddplan%d_workfracts" % i])
    assert plan.resolution == meta["resolution"]
    assert str(plan) == meta["text"]


def test_ddplan_subband_calls():
    obs = ddplan.Observation(64e-6, 1400.0, 300.0, 4096)
    plan = obs.gen_ddplan(0.0, 1000.0, 64, 0.5)
    (step,) = plan.DDsteps
    calls = step.subband_calls()
    assert len(calls) == step.numprepsub == 40
    assert all(len(d) == step.DMs_per_prepsub == 50 for _, d in calls)
    assert np.array_equal(np.concatenate([d for _, d in calls]), step.DMs)
    assert calls[0][0] == pytest.approx(0.5 * step.dsubDM)


# ---------------------------------------------------------------------------
# Full BASELINE grids pinned row-for-row against the reference's own bins
# (tests/golden/make_golden_grids.py records what Spectra.dedisperse /
# Spectra.subband hand to shift_channels, formats/spectra.py:126-130,247-250)
# ---------------------------------------------------------------------------
def _digest(row):
    import hashlib
    b = np.ascontiguousarray(np.asarray(row, dtype="<i4")).tobytes()
    return np.frombuffer(hashlib.blake2b(b, digest_size=8).digest(), dtype="<u8")[0]


@pytest.fixture(scope="module")
def grids():
    return np.load(os.path.join(GOLDEN, "golden_grids.npz"), allow_pickle=False)


def _check_rows(g, key, table):
    table = delays.to_int32(table)
    assert table.shape[0] == len(g[key + "_digest"])
    np.testing.assert_array_equal(table.max(axis=1), g[key + "_max"])
    got = np.array([_digest(r) for r in table], dtype="<u8")
    bad = np.nonzero(got != g[key + "_digest"])[0]
    assert bad.size == 0, "%s: %d rows differ from the reference (first %s)" % (key, bad.size,
                                                                                bad[:5])
    np.testing.assert_array_equal(table[0], g[key + "_row0"])
    np.testing.assert_array_equal(table[-1], g["%s_row%d" % (key, table.shape[0] - 1)])


@pytest.mark.parametrize("key,fkey", [("cfg0", "freqs1024"), ("cfg1", "freqs1024"),
                                      ("cfg3", "freqs4096"), ("ns", "freqs4096"),
                                      ("cfg4", "freqs4096")])
def test_baseline_grid_tables_match_reference(grids, key, fkey):
    """configs[0], [1], [3], [4] and the north-star grid: every row of the
    host sweep table equals the reference's dedisperse bins."""
    g = grids
    tab = delays.sweep_table(g[key + "_dms"], g[fkey], float(g[key + "_dt"]))
    _check_rows(g, key, tab)


def test_config2_two_stage_tables_match_reference(grids):
    """configs[2] (DDplan2b 4096 -> 64 subbands, res 0.5 ms): the plan's
    subband passes (subDM_k), the stage-1 tables (Spectra.subband bins) and
    the stage-2 tables (dedisperse bins on the subband centres) the
    DDplanExecutor builds are the reference's, row for row."""
    from pypulsar_amd.utils.ddplan import Observation
    g = grids
    freqs = g["freqs4096"]
    plan = Observation(64e-6, 1400.0, 300.0, 4096).gen_ddplan(0.0, 1000.0, 64, 0.5)
    assert len(plan.DDsteps) == 1
    st = plan.DDsteps[0]
    ds, ncall, per, dsub, lo, ddm = g["cfg2_meta"]
    assert (st.downsamp, st.numprepsub, st.DMs_per_prepsub) == (ds, ncall, per)
    calls = st.subband_calls()
    subdms = np.array([c[0] for c in calls])
    np.testing.assert_array_equal(subdms, g["cfg2s1_dms"])
    np.testing.assert_array_equal(np.concatenate([c[1] for c in calls]), g["cfg2s2_dms"])
    dt = 64e-6 * st.downsamp
    t1 = np.stack([delays.subband_bins(sd, freqs, dt, 64) for sd in subdms])
    _check_rows(g, "cfg2s1", t1)
    _, _, ctr = delays.subband_layout(freqs, 64)
    np.testing.assert_array_equal(ctr, g["cfg2_ctr"])
    t2 = delays.sweep_table(np.concatenate([c[1] for c in calls]), ctr, dt)
    _check_rows(g, "cfg2s2", t2)


def test_plan_model_ladder_covers_every_tiling():
    """The ladder grids of test_sweep_variant_ladder select every candidate
    tiling (pdd_sweep.hip), in order, under the plan-selection model."""
    import plan_model
    from oracle import spectra_oracle as orc
    from test_gpu_parity import LADDER
    freqs = band(32)
    for dtype, cands in (("f32", plan_model.F32), ("u8", plan_model.U8)):
        got = [plan_model.choose(orc.sweep_table(np.arange(64) * d, freqs, DT), dtype)
               for d in LADDER[dtype]]
        assert got == list(range(len(cands))), (dtype, got)


def test_plan_model_matches_kernel_tables():
    """tests/plan_model.py restates the candidate tables of pdd_sweep.hip."""
    import re
    import plan_model
    src = open(os.path.join(os.path.dirname(GOLDEN), "..", "pypulsar_amd", "csrc",
                            "pdd_sweep.hip")).read()
    for name, model in (("kF32Variants", plan_model.F32), ("kU8Variants", plan_model.U8)):
        body = src[src.index("static const Variant %s[] = {" % name):]
        body = body[:body.index("};")]
        # rows under #ifdef PDD_SWEEP_DEV are developer-build tilings only
        body = re.sub(r"#ifdef PDD_SWEEP_DEV.*?#endif", "", body, flags=re.S)
        rows = [tuple(int(v) if v not in ("true", "false") else int(v == "true")
                      for v in (x.strip() for x in m.split(",")))
                for m in re.findall(r"\{([-\w, ]+)\}", body)]
        assert rows == model, name
