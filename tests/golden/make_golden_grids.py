#!/usr/bin/env python
"""Pin the delay tables of every BASELINE.json grid against the reference.

RUN ONLY IN THE BUILD CONTAINER (it executes the read-only reference at
/root/reference the same way make_golden.py does; see that file for how).
For each grid the REFERENCE's own bins are recorded -- the argument
``Spectra.dedisperse`` / ``Spectra.subband`` pass to ``shift_channels``
(formats/spectra.py:126-130, 247-250) -- and stored as one 64-bit BLAKE2b
digest of the little-endian int32 row per DM trial (plus row maxima and a few
full rows), so the fixture stays small while every row is pinned bit-exact.

Grids (64 us, 1250-1550 MHz SIGPROC band, fch1 = hi - |foff|/2):
  configs[0]  1024 ch, DM 100                                (dt 64 us)
  configs[1]  1024 ch, 1024 DMs linspace(0, 1000)           (dt 64 us)
  configs[3]  4096 ch, 4096 DMs linspace(0, 1000)           (dt 64 us)
  north star  4096 ch, 2048 DMs linspace(0, 1000)           (dt 64 us)
  configs[4]  4096 ch, 2048 DMs linspace(0, 1000)           (dt 128 us: downsample 2)
  configs[2]  DDplan2b Observation(64us, 1400, 300, 4096).gen_ddplan(0, 1000, 64, 0.5):
              stage 1 = subband(64, subDM_k) bins of its 40 passes, stage 2 =
              dedisperse(dm) bins of all 2000 DMs on the 64 subband centres
              (dt = 64 us x the step's downsamp)

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_grids.py
"""
import hashlib
import os
import sys

sys.dont_write_bytecode = True
os.environ.setdefault("MPLBACKEND", "Agg")

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import band, load_reference  # noqa: E402


def row_digest(row):
    """64-bit BLAKE2b of a bins row as little-endian int32 (also used by the
    tests to compare the host tables)."""
    b = np.ascontiguousarray(np.asarray(row, dtype="<i4")).tobytes()
    return np.frombuffer(hashlib.blake2b(b, digest_size=8).digest(), dtype="<u8")[0]


def ref_dedisperse_bins(Spectra, freqs, dt, dm):
    """The bins the reference's Spectra.dedisperse(dm) hands shift_channels."""
    s = Spectra(freqs, dt, np.zeros((len(freqs), 4)))
    rec = []
    s.shift_channels = lambda bins, padval=0: rec.append(np.asarray(bins).copy())
    s.dedisperse(dm)
    return rec[0]


def ref_subband_bins(Spectra, freqs, dt, nsub, subdm):
    """The bins the reference's Spectra.subband(nsub, subdm) hands
    shift_channels (its data are not needed for the table)."""
    s = Spectra(freqs, dt, np.zeros((len(freqs), 4)))
    rec = []
    s.shift_channels = lambda bins, padval=0: rec.append(np.asarray(bins).copy())
    s.subband(nsub, subdm)
    return rec[0], np.asarray(s.freqs)


def pin(fx, key, rows, dms, keep=(0, -1)):
    rows = np.asarray(rows)
    fx[key + "_digest"] = np.array([row_digest(r) for r in rows], dtype="<u8")
    fx[key + "_max"] = rows.max(axis=1).astype(np.int64)
    fx[key + "_dms"] = np.asarray(dms, dtype=np.float64)
    for i in keep:
        fx["%s_row%d" % (key, i % len(rows))] = rows[i].astype(np.int32)


def main():
    spectra, ddplan, _ = load_reference()
    Spectra = spectra.Spectra
    fx = {}
    dt = 64e-6
    f1024, _, _ = band(1024)
    f4096, _, _ = band(4096)
    fx["freqs1024"] = f1024
    fx["freqs4096"] = f4096

    grids = [
        ("cfg0", f1024, dt, np.array([100.0])),
        ("cfg1", f1024, dt, np.linspace(0.0, 1000.0, 1024)),
        ("cfg3", f4096, dt, np.linspace(0.0, 1000.0, 4096)),
        ("ns", f4096, dt, np.linspace(0.0, 1000.0, 2048)),
        ("cfg4", f4096, 2 * dt, np.linspace(0.0, 1000.0, 2048)),
    ]
    for key, freqs, gdt, dms in grids:
        rows = [ref_dedisperse_bins(Spectra, freqs, gdt, dm) for dm in dms]
        pin(fx, key, rows, dms)
        fx[key + "_dt"] = np.array(gdt)
        print(key, len(rows), "rows, max bin", int(np.max(rows)), flush=True)

    # configs[2]: the DDplan2b plan and its two stages
    obs = ddplan.Observation(dt, 1400.0, 300.0, 4096, 0)
    plan = obs.gen_ddplan(0.0, 1000.0, 64, 0.5)
    assert len(plan.DDsteps) == 1
    st = plan.DDsteps[0]
    sdt = dt * st.downsamp
    ncall = int(st.numprepsub)
    per = int(st.DMs_per_prepsub)
    subdms = st.loDM + (np.arange(ncall) + 0.5) * st.dsubDM
    s1 = []
    ctr = None
    for sd in subdms:
        b, ctr = ref_subband_bins(Spectra, f4096, sdt, 64, sd)
        s1.append(b)
    pin(fx, "cfg2s1", s1, subdms)
    s2 = [ref_dedisperse_bins(Spectra, ctr, sdt, dm) for dm in st.DMs]
    pin(fx, "cfg2s2", s2, st.DMs)
    fx["cfg2_ctr"] = ctr
    fx["cfg2_meta"] = np.array([st.downsamp, ncall, per, st.dsubDM, st.loDM, st.dDM])
    print("cfg2: %d subDMs, %d DMs, ds %d" % (ncall, len(st.DMs), st.downsamp), flush=True)

    out = os.path.join(HERE, "golden_grids.npz")
    np.savez_compressed(out, **fx)
    print("wrote %s (%.2f MB)" % (out, os.path.getsize(out) / 1e6))


if __name__ == "__main__":
    main()
