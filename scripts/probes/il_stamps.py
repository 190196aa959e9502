# Per-wave cycle stamps of k_sweep_il (developer build, PDD_SWEEP_DEBUG=4):
# compute waves report (barrier wait, compute), loader waves (vmcnt wait,
# barrier wait, issue).  Usage (GPU box):
#   PDD_DEV_LIB=build/libpdd_dev.so PDD_SWEEP_DEBUG=4 python scripts/probes/il_stamps.py f32|u8
import sys
import numpy as np
import torch
sys.path.insert(0, '.')
from pypulsar_amd.sweep import DMSweep


def band(C, lo=1250.0, hi=1550.0):
    foff = -(hi - lo) / C
    return (hi + foff / 2.0) + foff * np.arange(C)


kind = sys.argv[1] if len(sys.argv) > 1 else "f32"
if kind == "f32":   # BASELINE configs[1]
    C, N, D, dt = 1024, 1 << 20, 1024, "f32"
elif kind == "ns":  # the north-star grid on a 2^20 block (factorised, groups of 2)
    C, N, D, dt = 4096, 1 << 20, 2048, "u8"
else:               # the configs[3] grid on a 2^20 block (factorised, groups of 4)
    C, N, D, dt = 4096, 1 << 20, 4096, "u8"
x = torch.randint(0, 256, (C, N), dtype=torch.uint8, device="cuda")
if dt == "f32":
    x = x.float()
sw = DMSweep(np.linspace(0, 1000, D), band(C), 64e-6, dtype=dt)
info = sw.info(1 if dt == "u8" else 0)
out = sw(x)
torch.cuda.synchronize()
nw = 16
st = out.view(-1)[: (out.numel() // (4 * nw)) * 4 * nw].view(-1, nw, 4).cpu().numpy()
comp = st[:, :, 3] == 1.0
blocks = int(np.argmax(~comp[:, 0])) if not comp[:, 0].all() else st.shape[0]
st = st[:blocks]
comp = comp[:blocks]
cw = st[comp]          # [n, 4]: 0, barrier, compute, 1
lw = st[~comp]         # [n, 4]: vmcnt, barrier, issue, 0
print(kind, info, "factor", sw.factor_info(1 if dt == "u8" else 0), "blocks", blocks)
print("compute waves: barrier %.0f  compute %.0f  -> barrier share %.3f"
      % (cw[:, 1].mean(), cw[:, 2].mean(), cw[:, 1].sum() / (cw[:, 1].sum() + cw[:, 2].sum())))
print("loader waves : vmcnt %.0f  barrier %.0f  issue %.0f"
      % (lw[:, 0].mean(), lw[:, 1].mean(), lw[:, 2].mean()))
# per wave slot: mean barrier wait / compute (compute waves) or vmcnt / barrier / issue
for w in range(nw):
    s = st[:, w]
    if comp[0, w]:
        print("  wave %2d compute: barrier %8.0f compute %8.0f" % (w, s[:, 1].mean(), s[:, 2].mean()))
    else:
        print("  wave %2d loader : vmcnt %8.0f barrier %8.0f issue %8.0f"
              % (w, s[:, 0].mean(), s[:, 1].mean(), s[:, 2].mean()))
