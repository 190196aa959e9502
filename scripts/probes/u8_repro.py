"""Reproduce abi_asan u8 mismatches: sweep via the C ABI vs a host sum."""
import ctypes, itertools, sys
import numpy as np, torch
sys.path.insert(0, '.')
from pypulsar_amd import _lib
from pypulsar_amd._lib import call, ptr

def run(C, N, D, kind, dtype, seed=0):
    rng = np.random.default_rng(seed)
    if kind == 'jit':
        tab = rng.integers(0, 2, size=(D, C)).astype(np.int32)
    elif kind == 'zero':
        tab = np.zeros((D, C), np.int32)
    elif kind == 'inc':
        tab = (np.arange(C)[None, :] * np.arange(D)[:, None] // max(1, C)).astype(np.int32)
    x = rng.integers(0, 256, size=(C, N), dtype=np.uint8)
    mx = max(0, int(tab.max()))
    n_out = N - mx
    if n_out <= 0:
        return 0, -1, None
    h = ctypes.c_void_p()
    code = _lib.U8 if dtype == 'u8' else _lib.F32
    _lib.check(_lib.lib().pdd_sweep_plan_create(tab.ctypes.data_as(ctypes.c_void_p), D, C, code, ctypes.byref(h)), 'plan')
    info = np.zeros(8, np.int64)
    _lib.lib().pdd_sweep_plan_info(h, info.ctypes.data_as(ctypes.c_void_p))
    xd = torch.from_numpy(x).cuda()
    if dtype == 'f32': xd = xd.float()
    out = torch.zeros((D, n_out), dtype=torch.float32, device='cuda')
    pv = torch.zeros(C, dtype=torch.float32, device='cuda')
    call('pdd_sweep_execute_ex', h, ptr(xd), N, N, 0, 0, 0, ptr(pv), ptr(out), n_out, n_out, 0.0, None)
    got = out.cpu().numpy()
    want = np.zeros((D, n_out))
    for d in range(D):
        for c in range(C):
            want[d] += x[c, tab[d, c]:tab[d, c] + n_out]
    bad = np.argwhere(got != want)
    _lib.lib().pdd_sweep_plan_destroy(h)
    return len(bad), info[7], (bad[:3].tolist(), got.flat[0], want.flat[0]) if len(bad) else None

for C, N, D, kind, dt in itertools.product([64, 96], [1, 4096, 5000, 8192, 5008], [1, 5, 40], ['jit', 'zero', 'inc'], ['u8', 'f32']):
    nb, v, ex = run(C, N, D, kind, dt)
    if nb or (N == 5000 and D == 1):
        print(C, N, D, kind, dt, 'variant', v, 'bad', nb, ex, flush=True)
print('done')
