#!/usr/bin/env python
"""Generate the golden fixtures that pin the oracle and the HIP path.

RUN ONLY IN THE BUILD CONTAINER (it imports the read-only reference at
/root/reference, which never travels to the GPU box).  Only the .npz/.json
fixtures this script writes are committed; no reference source, bytecode or
shim is copied into the repository.

How the reference is executed:
  * PRESTO is not installed, so a probe-only ``psr_utils`` module restating the
    three PRESTO functions the path uses (delay_from_DM, rotate, dm_smear) is
    written to a temp dir and put on sys.path.  Parity with PRESTO itself is
    therefore UNPINNED (PRESTO's version is not pinned by the reference).
  * ``formats/spectra.py`` is run from its own source text with exactly two
    Python-2 integer-division tokens patched to ``//`` (spectra.py:119 and
    spectra.py:345) -- the intended py2 semantics.
  * ``utils/DDplan2b.py`` is imported unmodified (MPLBACKEND=Agg).
  * ``filter`` of ``bin/zero_dm_filter.py:30-39`` is extracted via ``ast``.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
import ast
import importlib.util
import json
import os
import sys
import tempfile
import types

sys.dont_write_bytecode = True
os.environ.setdefault("MPLBACKEND", "Agg")

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))

# ---------------------------------------------------------------------------
# probe-only restatement of PRESTO's psr_utils (the three functions on path)
# ---------------------------------------------------------------------------
_PSR_UTILS_SHIM = '''
import numpy as Num
def delay_from_DM(DM, freq_emitted):
    if type(freq_emitted) == type(0.0):
        if freq_emitted > 0.0:
            return DM / (0.000241 * freq_emitted * freq_emitted)
        return 0.0
    return Num.where(freq_emitted > 0.0,
                     DM / (0.000241 * freq_emitted * freq_emitted), 0.0)
def rotate(arr, bins):
    bins = bins % len(arr)
    if bins == 0:
        return arr
    return Num.concatenate((arr[bins:], arr[:bins]))
def dm_smear(DM, BW, center_freq):
    return DM * BW / (0.0001205 * center_freq * center_freq * center_freq)
'''


def load_reference():
    shim_dir = tempfile.mkdtemp(prefix="pdd_probe_")
    with open(os.path.join(shim_dir, "psr_utils.py"), "w") as f:
        f.write(_PSR_UTILS_SHIM)
    sys.path.insert(0, shim_dir)

    # spectra.py with the two py2 floor-division tokens patched in memory
    src = open(os.path.join(REF, "formats", "spectra.py")).read()
    a = "nchan_per_sub = self.numchans/nsub"
    b = "new_num_spectra = self.numspectra/factor"
    assert src.count(a) == 1 and src.count(b) == 1
    src = src.replace(a, "nchan_per_sub = self.numchans//nsub")
    src = src.replace(b, "new_num_spectra = self.numspectra//factor")
    spectra = types.ModuleType("ref_spectra")
    exec(compile(src, "ref_spectra", "exec"), spectra.__dict__)

    spec = importlib.util.spec_from_file_location(
        "ref_ddplan", os.path.join(REF, "utils", "DDplan2b.py"))
    ddplan = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ddplan)

    zsrc = open(os.path.join(REF, "bin", "zero_dm_filter.py")).read()
    tree = ast.parse(zsrc)
    fn = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "filter"]
    assert len(fn) == 1
    zmod = ast.Module(body=fn, type_ignores=[])
    zns = {"np": np}
    exec(compile(zmod, "ref_zero_dm_filter", "exec"), zns)
    return spectra, ddplan, zns["filter"]


def band(C, descending=True, lo=1250.0, hi=1550.0):
    """SIGPROC frequencies exactly as filterbank.py:85 builds them."""
    foff = (hi - lo) / C
    if descending:
        fch1, foff = hi - foff / 2.0, -foff
    else:
        fch1 = lo + foff / 2.0
    return fch1 + foff * np.arange(C), fch1, foff


def u8_data(C, N, seed):
    rng = np.random.default_rng(seed)
    return np.clip(np.round(rng.normal(128, 16, size=(C, N))), 0, 255).astype(np.uint8)


def main():
    spectra, ddplan, zfilter = load_reference()
    Spectra = spectra.Spectra
    dt = 64e-6
    fx = {}
    meta = {"dt": dt, "cases": {}}

    def record_bins(s):
        rec = []
        orig = s.shift_channels

        def wrapped(bins, padval=0):
            rec.append(np.asarray(bins).copy())
            return orig(bins, padval)
        s.shift_channels = wrapped
        return rec

    # 1. delay-bin tables (bit-exact): dedisperse() bins for many DMs
    dms = np.array([0.0, 0.1, 1.0, 12.34, 50.0, 100.0, 333.3, 567.89, 1000.0, 2000.0])
    for C in (64, 1024, 4096):
        for desc in (True, False):
            freqs, _, _ = band(C, desc)
            rows = []
            for dm in dms:
                s = Spectra(freqs, dt, np.zeros((C, 4)))
                rec = record_bins(s)
                s.dedisperse(dm)
                rows.append(rec[0])
            key = "bins_C%d_%s" % (C, "desc" if desc else "asc")
            fx[key] = np.array(rows, dtype=np.int64)
            fx[key + "_freqs"] = freqs
    fx["bins_dms"] = dms

    # uniform 0..1000 grid on the config-2 band (1024 DMs)
    freqs, _, _ = band(1024, True)
    grid = np.linspace(0.0, 1000.0, 1024)
    rows = []
    for dm in grid[::17]:
        s = Spectra(freqs, dt, np.zeros((1024, 4)))
        rec = record_bins(s)
        s.dedisperse(dm)
        rows.append(rec[0])
    fx["bins_grid_dms"] = grid[::17]
    fx["bins_grid"] = np.array(rows, dtype=np.int64)

    # 2. dedisperse outputs, all pad modes x trim, incl. |shift|>=N & negative shifts
    C, N = 16, 256
    x = u8_data(C, N, 1)
    fx["dd_x"] = x
    for desc in (True, False):
        freqs, _, _ = band(C, desc)
        tag = "desc" if desc else "asc"
        fx["dd_freqs_" + tag] = freqs
        for pi, pad in enumerate([0, 3.5, "mean", "median", "rotate"]):
            for trim in (False, True):
                for dm in (100.0, 3000.0):
                    s = Spectra(freqs, dt, x)
                    s.dedisperse(dm, padval=pad, trim=trim)
                    k = "dd_%s_p%d_t%d_dm%d" % (tag, pi, int(trim), int(dm))
                    fx[k] = s.data
                # two-step: dedisperse at 100 then at 50 (negative shifts)
                s = Spectra(freqs, dt, x)
                s.dedisperse(100.0, padval=pad)
                s.dedisperse(50.0, padval=pad, trim=trim)
                fx["dd2_%s_p%d_t%d" % (tag, pi, int(trim))] = s.data
    meta["pads"] = [0, 3.5, "mean", "median", "rotate"]

    # 3. subband: nsub in {1, 8, C} x subdm in {None, 0, 50} x pad {0, mean}, both band orders
    C, N = 32, 256
    x = u8_data(C, N, 2)
    fx["sb_x"] = x
    for desc in (True, False):
        freqs, _, _ = band(C, desc)
        tag = "desc" if desc else "asc"
        fx["sb_freqs_" + tag] = freqs
        for nsub in (1, 8, C):
            for si, subdm in enumerate([None, 0.0, 50.0, 400.0]):
                for pi, pad in enumerate([0, "mean"]):
                    s = Spectra(freqs, dt, x)
                    rec = record_bins(s)
                    s.subband(nsub, subdm, padval=pad)
                    k = "sb_%s_n%d_s%d_p%d" % (tag, nsub, si, pi)
                    fx[k] = s.data
                    fx[k + "_freqs"] = s.freqs
                    if rec:
                        fx[k + "_bins"] = rec[0]
                    assert s.dm == 0
        # subband then dedisperse (waterfaller chain, padval='mean', trim=True)
        s = Spectra(freqs, dt, x)
        s.subband(8, 100.0, padval="mean")
        s.dedisperse(100.0, padval="mean", trim=True)
        fx["sbdd_%s" % tag] = s.data
    meta["subdms"] = [None, 0.0, 50.0, 400.0]

    # 4. downsample with remainders
    C, N = 8, 1000
    x = u8_data(C, N, 3)
    fx["ds_x"] = x
    freqs, _, _ = band(C)
    for f in (1, 3, 4, 8, 7):
        s = Spectra(freqs, dt, x)
        s.downsample(f)
        fx["ds_f%d" % f] = s.data
        fx["ds_f%d_dt" % f] = np.array(s.dt)
        fx["ds_f%d_n" % f] = np.array(s.numspectra)

    # 5. trim (b>0 and b<0; b<0 keeps the reference's numspectra bug)
    s = Spectra(freqs, dt, x, starttime=1.0)
    s.trim(10)
    fx["trim_pos"] = s.data
    fx["trim_pos_meta"] = np.array([s.numspectra, s.starttime])
    s = Spectra(freqs, dt, x, starttime=1.0)
    s.trim(-10)
    fx["trim_neg"] = s.data
    fx["trim_neg_meta"] = np.array([s.numspectra, s.starttime])

    # 6. zero-DM filter per spectrum: uint8 / uint16 / float32, incl. ties
    rng = np.random.default_rng(4)
    z8 = rng.integers(0, 256, size=(64, 96), dtype=np.uint8)
    z8[0, :4] = [10, 200, 100, 3]  # documented probe vector when C=4
    z16 = rng.integers(0, 65536, size=(64, 96), dtype=np.uint16)
    zf = rng.normal(0, 10, size=(64, 96)).astype(np.float32)
    tie = np.zeros((4, 4), dtype=np.uint8)
    tie[0] = [1, 2, 3, 4]      # mean 2.5 -> 2 (half-even)
    tie[1] = [2, 3, 4, 5]      # mean 3.5 -> 4
    tie[2] = [0, 0, 0, 2]      # mean 0.5 -> 0
    tie[3] = [255, 255, 255, 1]
    probe = np.array([[10, 200, 100, 3]], dtype=np.uint8)
    for name, arr in (("u8", z8), ("u16", z16), ("f32", zf), ("tie", tie), ("probe", probe)):
        fx["zd_in_" + name] = arr
        fx["zd_out_" + name] = np.array([zfilter(row) for row in arr])

    # 7. DDplan2b step tables
    plans = [
        dict(dt=64e-6, fctr=1400.0, BW=300.0, numchan=1024, numsamp=0, lo=0.0, hi=1000.0, nsub=0, res=0.0),
        dict(dt=64e-6, fctr=1400.0, BW=300.0, numchan=4096, numsamp=0, lo=0.0, hi=1000.0, nsub=64, res=0.5),
        dict(dt=64e-6, fctr=1400.0, BW=300.0, numchan=4096, numsamp=0, lo=0.0, hi=1000.0, nsub=64, res=0.0),
        dict(dt=64e-6, fctr=1400.0, BW=300.0, numchan=1024, numsamp=0, lo=0.0, hi=1000.0, nsub=32, res=1.0),
        dict(dt=81.92e-6, fctr=1375.0, BW=322.6, numchan=960, numsamp=2 ** 20, lo=10.0, hi=2000.0, nsub=0, res=0.3),
        dict(dt=64e-6, fctr=350.0, BW=100.0, numchan=4096, numsamp=0, lo=0.0, hi=500.0, nsub=128, res=0.0),
    ]
    meta["ddplans"] = []
    for i, p in enumerate(plans):
        obs = ddplan.Observation(p["dt"], p["fctr"], p["BW"], p["numchan"], p["numsamp"])
        plan = obs.gen_ddplan(p["lo"], p["hi"], p["nsub"], p["res"])
        steps = []
        for st in plan.DDsteps:
            d = dict(loDM=st.loDM, hiDM=st.hiDM, dDM=st.dDM, downsamp=int(st.downsamp),
                     numDMs=int(st.numDMs), dsubDM=st.dsubDM, numprepsub=int(st.numprepsub),
                     DMs_per_prepsub=int(getattr(st, "DMs_per_prepsub", 0)),
                     BW_smearing=st.BW_smearing, sub_smearing=st.sub_smearing)
            steps.append(d)
            fx["ddplan%d_step%d_DMs" % (i, len(steps) - 1)] = st.DMs
            fx["ddplan%d_step%d_totsmear" % (i, len(steps) - 1)] = st.tot_smear
        fx["ddplan%d_workfracts" % i] = plan.work_fracts
        meta["ddplans"].append(dict(params=p, steps=steps, resolution=plan.resolution,
                                    text=str(plan)))

    # 8. sweep pins: per-DM (dedisperse(trim=True) + channel sum) compositions
    C, N = 64, 4096
    x = u8_data(C, N, 5)
    fx["sw_x"] = x
    freqs, _, _ = band(C)
    fx["sw_freqs"] = freqs
    sdms = np.linspace(0.0, 250.0, 24)
    fx["sw_dms"] = sdms
    rows = []
    lens = []
    for dm in sdms:
        s = Spectra(freqs, dt, x)
        s.dedisperse(dm, padval=0, trim=True)
        rows.append(s.data.sum(axis=0))
        lens.append(s.numspectra)
    L = min(lens)
    fx["sw_plane"] = np.array([r[:L] for r in rows])
    fx["sw_lens"] = np.array(lens)
    # full-length (trim=False) rows with pad 0 and with 'mean'
    for pi, pad in enumerate([0, "mean"]):
        rows = []
        for dm in sdms:
            s = Spectra(freqs, dt, x)
            s.dedisperse(dm, padval=pad, trim=False)
            rows.append(s.data.sum(axis=0))
        fx["sw_plane_full_p%d" % pi] = np.array(rows)

    # two-stage subband sweep (per call: subband(nsub, subDM) then dedisperse(dm, trim=True))
    nsub = 8
    subDM = 40.0
    sdms2 = np.arange(30.0, 50.0, 1.0)
    rows = []
    lens = []
    for dm in sdms2:
        s = Spectra(freqs, dt, x)
        s.subband(nsub, subDM, padval=0)
        s.dedisperse(dm, padval=0, trim=True)
        rows.append(s.data.sum(axis=0))
        lens.append(s.numspectra)
    L = min(lens)
    fx["sw2_dms"] = sdms2
    fx["sw2_plane"] = np.array([r[:L] for r in rows])
    fx["sw2_lens"] = np.array(lens)
    meta["sw2"] = dict(nsub=nsub, subDM=subDM)

    # 9. downsample-then-dedisperse (a DDplan step with downsamp 4)
    s = Spectra(freqs, dt, x)
    s.downsample(4)
    s.dedisperse(200.0, trim=True)
    fx["dsdd_series"] = s.data.sum(axis=0)
    fx["dsdd_dt"] = np.array(s.dt)

    np.savez_compressed(os.path.join(OUT, "golden.npz"), **fx)
    with open(os.path.join(OUT, "golden_meta.json"), "w") as f:
        json.dump(meta, f, indent=1, default=float)
    tot = os.path.getsize(os.path.join(OUT, "golden.npz"))
    print("wrote %d arrays, %.2f MB" % (len(fx), tot / 1e6))


if __name__ == "__main__":
    main()
