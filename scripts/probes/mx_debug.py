import sys, numpy as np, torch
sys.path.insert(0, '.')
import __graft_entry__ as g; g.build()
from pypulsar_amd.sweep import DMSweep
from oracle import spectra_oracle as orc
def band(C, lo=1250.0, hi=1550.0):
    foff = -(hi - lo) / C
    return (hi + foff / 2.0) + foff * np.arange(C)
DT = 64e-6
def run(C, N, dms, x, tag):
    xd = torch.from_numpy(x).cuda()
    sw = DMSweep(dms, band(C), DT, dtype="u8")
    v = sw.info(1)["variant"]
    plane = sw(xd).cpu().numpy().astype(np.float64)
    tab = orc.sweep_table(dms, band(C), DT)
    want = orc.sweep_plane(x.astype(np.float64), tab)
    ok = np.array_equal(plane, want)
    print("%s variant %d ok %s maxbin %d" % (tag, v, ok, tab.max()), flush=True)
    if not ok:
        d = plane - want
        bad = np.argwhere(d != 0)
        print("  nbad %d of %d; first %s" % (len(bad), d.size, bad[:8].tolist()))
        r = bad[0][0]
        print("  row", r, "got", plane[r, :12].tolist())
        print("  row", r, "want", want[r, :12].tolist())
        print("  diff row0 cols 0..40:", d[r, :40].tolist())
    sw.close()
C, N = 64, 4096
x1 = np.ones((C, N), np.uint8)
run(C, N, np.zeros(16), x1, "ones dm0")
x = np.random.default_rng(1).integers(0, 256, (C, N), dtype=np.uint8)
run(C, N, np.zeros(16), x, "rand dm0")
xr = np.tile(np.arange(N, dtype=np.int64) % 251, (C, 1)).astype(np.uint8)
run(C, N, np.zeros(16), xr, "ramp dm0")
run(C, N, np.linspace(0, 5, 16), xr, "ramp dm0-5")
run(C, N, np.linspace(0, 5, 16), x, "rand dm0-5")
run(128, N, np.linspace(0, 50, 40), np.random.default_rng(2).integers(0, 256, (128, N), dtype=np.uint8), "rand C128 dm0-50")
