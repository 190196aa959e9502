"""Diagnostic: per-wave cycle split of the interleaved sweep (PDD_SWEEP_DEBUG=4,
timing-only: the plane is overwritten with stamps).  Usage: il_stamps.py V..."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import __graft_entry__ as g  # noqa: E402

g.build()
from pypulsar_amd.sweep import DMSweep  # noqa: E402

C, N, D = 1024, 1 << 20, 1024
foff = -300.0 / C
freqs = 1550 + foff / 2 + foff * np.arange(C)
dms = np.linspace(0, 1000, D)
x = torch.randn(C, N, device="cuda")
for v in sys.argv[1:]:
    os.environ["PDD_SWEEP_VARIANT"] = v
    os.environ["PDD_SWEEP_DEBUG"] = "4"
    sw = DMSweep(dms, freqs, 64e-6)
    out = sw(x)
    out.zero_()
    sw(x, out=out)
    torch.cuda.synchronize()
    info = sw.info()
    st = out.flatten()[: 4 * 400000].view(-1, 4).cpu().numpy().astype(np.float64)
    st = st[np.abs(st).sum(axis=1) > 0]
    comp = st[st[:, 3] == 1]
    load = st[st[:, 3] == 0]
    steps = C / info["chans_per_chunk"]
    print("v=%s DB=%d cc=%d | compute waves %d: poll %.0f compute %.0f cyc/step | "
          "loader waves %d: vmwait %.0f poll %.0f issue %.0f cyc/step"
          % (v, info["dms_per_block"], info["chans_per_chunk"], len(comp), comp[:, 1].mean() / steps,
             comp[:, 2].mean() / steps, len(load), load[:, 0].mean() / steps,
             load[:, 1].mean() / steps, load[:, 2].mean() / steps))
    sw.close()
