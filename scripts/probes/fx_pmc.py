# Two factorised 8-bit sweep launches (planner's choice) on a 4096 x N block at
# the configs[3] (D=4096) or north-star (D=2048) grid, for rocprofv3 PMC passes.
#   python scripts/probes/fx_pmc.py [D] [log2 N]
import sys
import numpy as np
import torch
sys.path.insert(0, '.')
from pypulsar_amd.sweep import DMSweep


def band(C, lo=1250.0, hi=1550.0):
    foff = -(hi - lo) / C
    return (hi + foff / 2.0) + foff * np.arange(C)


D = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N = 1 << (int(sys.argv[2]) if len(sys.argv) > 2 else 20)
C = 4096
x = torch.randint(0, 256, (C, N), dtype=torch.uint8, device="cuda")
sw = DMSweep(np.linspace(0, 1000, D), band(C), 64e-6, dtype="u8")
out = sw(x)
torch.cuda.synchronize()
out = sw(x, out=out)
torch.cuda.synchronize()
print("ok", sw.factor_info(), sw.info(1))
