"""Diagnostic: per-wave cycle split of the ring sweep kernel (PDD_SWEEP_DEBUG=4).
Timing-only build (outputs are overwritten with stamps)."""
import os, sys, time
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import __graft_entry__ as g
g.build()
from pypulsar_amd.sweep import DMSweep
C, N, D = 1024, 1 << 20, 1024
foff = -300.0 / C
freqs = 1550 + foff / 2 + foff * np.arange(C)
dms = np.linspace(0, 1000, D)
x = torch.randn(C, N, device="cuda")
for dbg in [int(a) for a in sys.argv[1:]] or [4]:
    os.environ["PDD_SWEEP_DEBUG"] = str(dbg)
    sw = DMSweep(dms, freqs, 64e-6)
    out = sw(x)
    torch.cuda.synchronize()
    t = time.perf_counter(); sw(x, out=out); torch.cuda.synchronize(); el = time.perf_counter() - t
    info = sw.info()
    if dbg & 4:
        nw = 8
        nblk = (out.shape[1] + 1023) // 1024 * ((D + 31) // 32)
        st = out.flatten()[: nblk * nw * 4].view(-1, 4).cpu().numpy().astype(np.float64)
        tot = st.sum(axis=1)
        print("dbg=%d %.1f ms  P=%d  per-wave cycles: wait %.0f  barrier %.0f  issue %.0f  compute %.0f  (total %.0f; per step %.0f)"
              % (dbg, el * 1e3, info["chans_per_chunk"], *st.mean(axis=0), tot.mean(), tot.mean() / C))
    else:
        print("dbg=%d %.1f ms P=%d" % (dbg, el * 1e3, info["chans_per_chunk"]))
