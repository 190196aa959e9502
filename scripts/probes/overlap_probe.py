# Stage-1 / stage-2 overlap on CU-partitioned streams (pdd_sweep_execute_stage,
# pdd_stream_create_cu_mask): one factorised launch of the configs[3] /
# north-star grid (4096 ch, 1.04 M columns per launch), timed
#   full   : stage 1 + stage 2 on the default stream (today's launch);
#   s1/s2  : each stage alone on its CU subset;
#   overlap: stage 2 of block k (buffer A, big CU set) concurrently with
#            stage 1 of block k+1 (buffer B, small CU set), per block.
# Usage (GPU box): python scripts/probes/overlap_probe.py [config3|northstar] [m1 ...]
import sys, time
import numpy as np
import torch
sys.path.insert(0, '.')
from pypulsar_amd.sweep import DMSweep, cu_masked_stream, cu_stream_release


def band(C, lo=1250.0, hi=1550.0):
    foff = -(hi - lo) / C
    return (hi + foff / 2.0) + foff * np.arange(C)


cfg = sys.argv[1] if len(sys.argv) > 1 else "config3"
ms_small = [int(a) for a in sys.argv[2:]] or [16, 32]
C, D = 4096, 4096 if cfg == "config3" else 2048
sw = DMSweep(np.linspace(0, 1000, D), band(C), 64e-6, dtype="u8")
n_cols = 1044950
N = n_cols + sw.max_bin
x = torch.randint(0, 256, (C, N), dtype=torch.uint8, device="cuda")
out = torch.empty((D, n_cols), dtype=torch.float32, device="cuda")
nbytes = sw.pattern_bytes(n_cols)
print(cfg, "factor", sw.factor_info(), "skew", sw.skew_info(), "pattern GB %.1f" % (nbytes / 1e9), flush=True)
A = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
B = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
ref = torch.empty_like(out)
sw(x, out=ref, n_out=n_cols)


def timed(fn, reps=3):
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) * 1e3
        best = el if best is None else min(best, el)
    return best


t_full = timed(lambda: sw.sweep_pieces_stage(x, N, 0, 0, n_cols, out, A, 3))
assert torch.equal(out, ref)
print("full (stage 1 + 2, default stream): %.2f ms" % t_full, flush=True)
t1 = timed(lambda: sw.sweep_pieces_stage(x, N, 0, 0, n_cols, None, A, 1))
t2 = timed(lambda: sw.sweep_pieces_stage(x, N, 0, 0, n_cols, out, A, 2))
print("all CUs: stage 1 %.2f ms, stage 2 %.2f ms" % (t1, t2), flush=True)
for m in ms_small:
    # mask bit i -> XCC i % 8 (the driver spreads a queue's CU mask over
    # the XCCs round robin): the top m bits are m / 8 CUs of every XCC
    small = list(range(256 - m, 256))
    big = list(range(256 - m))
    s1 = cu_masked_stream(small)
    s2 = cu_masked_stream(big)
    ta = timed(lambda: sw.sweep_pieces_stage(x, N, 0, 0, n_cols, None, B, 1, stream=s1))
    tb = timed(lambda: sw.sweep_pieces_stage(x, N, 0, 0, n_cols, out, A, 2, stream=s2))
    sw.sweep_pieces_stage(x, N, 0, 0, n_cols, None, A, 1)
    torch.cuda.synchronize()

    def both():
        sw.sweep_pieces_stage(x, N, 0, 0, n_cols, out, A, 2, stream=s2)
        sw.sweep_pieces_stage(x, N, 0, 0, n_cols, None, B, 1, stream=s1)
    tc = timed(both)
    assert torch.equal(out, ref)
    print("m=%d CUs for stage 1: stage 1 alone %.2f ms, stage 2 alone on %d CUs %.2f ms, "
          "concurrent %.2f ms (serial today %.2f)" % (m, ta, 256 - m, tb, tc, t1 + t2), flush=True)
    cu_stream_release(s1)
    cu_stream_release(s2)
