"""The abi_asan driver's table shape through the Python/ctypes path."""
import ctypes, sys
import numpy as np, torch
sys.path.insert(0, '.')
from pypulsar_amd import _lib
from pypulsar_amd._lib import call, ptr

def run(C, N, D, span, dtype, seed):
    rng = np.random.default_rng(seed)
    d = np.arange(D)[:, None]; c = np.arange(C)[None, :]
    tab = ((d * span) // max(1, D) * (C - c) // C + rng.integers(0, 2, (D, C)) * (span > 0)).astype(np.int32)
    x = rng.integers(0, 256, size=(C, N), dtype=np.uint8)
    n_out = N - max(0, int(tab.max()))
    h = ctypes.c_void_p()
    code = _lib.U8 if dtype else _lib.F32
    _lib.check(_lib.lib().pdd_sweep_plan_create(tab.ctypes.data_as(ctypes.c_void_p), D, C, code, ctypes.byref(h)), 'plan')
    xd = torch.from_numpy(x).cuda()
    if not dtype: xd = xd.float()
    out = torch.zeros((D, n_out), dtype=torch.float32, device='cuda')
    pv = torch.zeros(C, dtype=torch.float32, device='cuda')
    call('pdd_sweep_execute_ex', h, ptr(xd), N, N, 0, 0, 0, ptr(pv), ptr(out), n_out, n_out, 0.0, None)
    got = out.cpu().numpy()
    want = np.zeros((D, n_out))
    for dd in range(D):
        for cc in range(C):
            want[dd] += x[cc, tab[dd, cc]:tab[dd, cc] + n_out]
    _lib.lib().pdd_sweep_plan_destroy(h)
    return int((got != want).sum()), got.flat[0], want.flat[0]

for case in [(96, 5000, 5, 40, 0), (96, 5000, 5, 40, 1), (96, 5000, 1, 900, 0), (96, 5000, 57, 900, 1),
             (64, 5000, 5, 900, 1), (96, 4096, 5, 40, 0)]:
    for rep in range(4):
        print(case, rep, run(*case, seed=rep), flush=True)
