# One 8-bit sweep launch at the config-3 grid on a 4096 x 2^20 block (for PMC passes).
import sys, numpy as np, torch
sys.path.insert(0, '.')
from pypulsar_amd.sweep import DMSweep
def band(C, lo=1250.0, hi=1550.0):
    foff = -(hi - lo) / C
    return (hi + foff / 2.0) + foff * np.arange(C)
C, N, D = 4096, 1 << 20, 4096
x = torch.randint(0, 256, (C, N), dtype=torch.uint8, device="cuda")
sw = DMSweep(np.linspace(0, 1000, D), band(C), 64e-6, dtype="u8")
out = sw(x)
torch.cuda.synchronize()
out = sw(x, out=out)
torch.cuda.synchronize()
print("ok", sw.info(1))
