import sys, numpy as np, torch
sys.path.insert(0, '.')
import __graft_entry__ as g; g.build()
from pypulsar_amd.sweep import DMSweep
from oracle import spectra_oracle as orc
def band(C, lo=1250.0, hi=1550.0):
    foff = -(hi - lo) / C
    return (hi + foff / 2.0) + foff * np.arange(C)
C, N, D, DT = 32, 49152, 64, 64e-6
x = np.random.default_rng(21).integers(0, 256, (C, N), dtype=np.uint8)
xd = torch.from_numpy(x).cuda()
for ddm in [0.5, 1.0, 1.3, 1.6, 2.0, 2.5, 3.0, 4.0, 5.0, 7.0, 12.0, 25.0, 40.0]:
    dms = np.arange(D) * ddm
    sw = DMSweep(dms, band(C), DT, dtype="u8")
    v = sw.info(1)
    plane = sw(xd).cpu().numpy().astype(np.float64)
    want = orc.sweep_plane(x.astype(np.float64), orc.sweep_table(dms, band(C), DT))
    ok = np.array_equal(plane, want)
    bad = np.argwhere(plane != want)
    print("dDM %5.2f variant %d lds %d ok %s %s" % (ddm, v["variant"], v["lds_bytes"], ok, bad[:3].tolist() if not ok else ""), flush=True)
    sw.close()
