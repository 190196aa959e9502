"""Single-pulse search (pdd_sp_chunk_stats + pdd_sp_search) on the GPU against
the float64 oracle (oracle/search_oracle.py) and end to end behind the sweep.
Tolerance: S/N within 1e-4 relative (f32 prefix sums vs float64); (start,
width) bit-exact except where the oracle's best and runner-up are closer
than 1e-4 (a float near-tie)."""
import numpy as np
import pytest

from conftest import band, u8_data
from oracle import search_oracle as so

pytestmark = pytest.mark.gpu
WIDTHS = (1, 2, 3, 4, 6, 9, 14, 20, 30, 45, 70, 100, 150)
DT = 64e-6


def _check(gpu_c, ora, margins, thr):
    og = {(d, t // 1024): (t, w, s, m) for (d, t, w, s), m in zip(ora, margins)}
    gg = {(int(r), int(t) // 1024): (int(t), int(w), float(s))
          for r, t, w, s in zip(gpu_c["row"], gpu_c["Sample"], gpu_c["Downfact"], gpu_c["Sigma"])}
    for k in set(og) | set(gg):
        if k in og and k in gg:
            t, w, s, m = og[k]
            assert abs(gg[k][2] - s) <= 1e-4 * max(1.0, abs(s)), (k, gg[k], og[k])
            if m > 1e-4 * abs(s):
                assert gg[k][:2] == (t, w), (k, gg[k], og[k])
        else:  # only allowed at the threshold
            s = og[k][2] if k in og else gg[k][2]
            assert abs(s - thr) <= 1e-4 * abs(thr), (k, s)


@pytest.mark.parametrize("D,n,L", [(7, 5000, 1000), (3, 1024, 256), (2, 777, 1000),
                                   (1, 100, 30), (4, 3 * 1024 + 1, 1024)])
def test_search_vs_oracle(gpu, D, n, L):
    import torch
    from pypulsar_amd.search import SinglePulseSearch
    rng = np.random.default_rng(D * 1000 + n)
    x = rng.normal(0, 1, (D, n))
    for d in range(D):  # a few pulses of random width
        for _ in range(2):
            w = int(rng.integers(1, 60))
            t = int(rng.integers(0, max(1, n - w)))
            x[d, t:t + w] += rng.uniform(0.5, 4.0)
    x[0, n // 3:n // 3 + 3] += 8.0  # at least one clear detection
    x = x.astype(np.float32)
    thr = 4.0
    sp = SinglePulseSearch(threshold=thr, widths=WIDTHS, detrendlen=L)
    got = sp(torch.from_numpy(x).cuda(), dms=np.arange(D) * 1.0, dt=1e-3)
    ora, margins = so.search(x.astype(np.float64), WIDTHS, thr, L)
    assert len(ora) > 0
    _check(got, ora, margins, thr)


def test_search_strided_constant_and_overflow(gpu):
    import torch
    from pypulsar_amd.search import SinglePulseSearch
    rng = np.random.default_rng(5)
    big = torch.zeros((4, 3000), device="cuda")
    big[:, :2500] = torch.from_numpy(rng.normal(0, 1, (4, 2500)).astype(np.float32)).cuda()
    big[1, 600:610] += 5.0
    big[2, :2500] = 7.0  # constant row: std 0 -> z 0 -> no candidate
    view = big[:, :2500]  # row stride 3000
    sp = SinglePulseSearch(threshold=5.0, detrendlen=500)
    got = sp(view, dms=[1.0, 2.0, 3.0, 4.0], dt=1e-3, t0=10)
    assert 2 not in set(got["row"])
    hit = got[got["row"] == 1]
    assert len(hit) == 1 and abs(int(hit["Sample"][0]) - 610) <= 10
    ora, m = so.search(view.cpu().numpy().astype(np.float64), sp.widths, 5.0, 500)
    got0 = got.copy()
    got0["Sample"] -= 10
    _check(got0, ora, m, 5.0)
    small = SinglePulseSearch(threshold=-100.0, detrendlen=500, max_cands=3)
    with pytest.raises(RuntimeError):
        small(view, dms=[1.0, 2.0, 3.0, 4.0], dt=1e-3)


def test_sweep_then_search_finds_dispersed_pulse(gpu):
    """End to end: a dispersed pulse injected at DM 120 into an 8-bit
    filterbank -> DMSweep plane -> search: the brightest candidate sits at the
    injected DM (grid step 2) and arrival sample."""
    import torch
    from pypulsar_amd.delays import delay_from_DM
    from pypulsar_amd.search import SinglePulseSearch
    from pypulsar_amd.sweep import DMSweep
    C, N, dt = 256, 1 << 15, 64e-6
    freqs = band(C)
    x = u8_data(C, N, 9).astype(np.int32)
    dm0, t0, w = 120.0, 9000, 8
    d = delay_from_DM(dm0, freqs) - delay_from_DM(dm0, freqs.max())
    bins = np.round(d / dt).astype(int)
    for c in range(C):
        x[c, t0 + bins[c]:t0 + bins[c] + w] += 12
    x = np.clip(x, 0, 255).astype(np.uint8)
    dms = np.arange(0, 300, 2.0)
    sw = DMSweep(dms, freqs, dt, dtype="u8")
    plane = sw(torch.from_numpy(x).cuda(), trim=True)
    cands = SinglePulseSearch(threshold=8.0)(plane, dms, dt)
    best = cands[np.argmax(cands["Sigma"])]
    assert abs(best["DM"] - dm0) <= 2.0 and abs(int(best["Sample"]) - t0) <= w
    assert best["Sigma"] > 20


@pytest.mark.parametrize("nchunks,last,nplanes", [(4, 8192, 0), (3, 3000, 0), (5, 8192, 2)])
def test_streaming_search_equals_one_shot(gpu, nchunks, last, nplanes):
    """StreamingSearch (blocks searched one behind the sweep, rows continued
    into the next block's plane) finds exactly the candidates of a one-shot
    search of the whole stream's plane, including pulses straddling block
    boundaries."""
    import torch
    from pypulsar_amd import _lib
    from pypulsar_amd._lib import call, ptr, stream_ptr
    from pypulsar_amd.search import SinglePulseSearch, StreamingSearch
    from pypulsar_amd.sweep import DMSweep
    C, block, ds = 64, 8192, 2
    freqs = band(C)
    dms = np.linspace(0.0, 60.0, 24)
    N = block * (nchunks - 1) + last
    rng = np.random.default_rng(3)
    x = np.clip(np.round(rng.normal(128, 16, (N, C))), 0, 255).astype(np.uint8)
    # bursts dispersed at DM 30 (zero-DM would remove undispersed ones), the
    # first two arriving (at the top of the band) just before block seams
    from pypulsar_amd.delays import delay_from_DM
    bins = np.round((delay_from_DM(30.0, freqs) - delay_from_DM(30.0, freqs.max())) / DT)
    xi = x.astype(np.int32)
    for t in (block - 20, 2 * block - 3, block + 1000):
        for c in range(C):
            b = t + int(bins[c])
            xi[b:b + 12, c] += 40
    x = np.clip(xi, 0, 255).astype(np.uint8)
    widths = (1, 2, 4, 8, 16, 32)
    ss = StreamingSearch(dms, freqs, DT, block=block, downsamp=ds, threshold=5.0, widths=widths,
                         detrendlen=1024)
    chunks = [torch.from_numpy(x[i:i + block]).pin_memory() for i in range(0, N, block)]
    # nplanes = 2: the minimum preallocated rotation (block j -> planes[j % 2])
    planes = ([torch.empty((len(dms), block // ds), dtype=torch.float32, device="cuda")
               for _ in range(nplanes)] if nplanes else None)
    got = np.concatenate(list(ss(chunks, planes=planes)))
    ss.close()
    xd = torch.from_numpy(x).cuda()
    f32 = torch.empty((C, N // ds), dtype=torch.float32, device="cuda")
    call("pdd_zdm_downsample", ptr(xd), _lib.U8, N, C, C, ds, 1, ptr(f32), f32.stride(0),
         stream_ptr())
    plane = DMSweep(dms, freqs, DT * ds)(f32)
    want = SinglePulseSearch(threshold=5.0, widths=widths, detrendlen=1024)(plane, dms, DT * ds)
    assert len(want) > 0
    key = lambda r: sorted(zip(r["row"], r["Sample"], r["Downfact"]))
    assert key(got) == key(want)
    np.testing.assert_array_equal(np.sort(got["Sigma"]), np.sort(want["Sigma"]))


def test_search_snr_pinned_to_reference_smooth(gpu):
    """Device search on the rows of tests/golden/golden_pulse.npz (already
    chunk-normalised, float32 values) against the reference's own
    Pulse.smooth (formats/pulse.py:217-241): every 1024-start window's best
    S/N over the search widths equals the maximum of the reference's smoothed
    profiles over the same starts (interior: Pulse.smooth[t + w//2]) within
    1e-4, and the detections match."""
    import os
    import torch
    from pypulsar_amd.search import SinglePulseSearch
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                             "golden_pulse.npz"), allow_pickle=False)
    z = g["z"]
    R, n = z.shape
    widths = tuple(int(w) for w in g["widths"])
    best = np.full((R, -(-n // 1024)), -np.inf)
    for w in widths:
        s = g["smooth_w%d" % w][:, w // 2:w // 2 + n - w + 1]    # start t -> Pulse.smooth[t + w//2]
        pad = best.shape[1] * 1024 - s.shape[1]
        s = np.concatenate([s, np.full((R, pad), -np.inf)], axis=1).reshape(R, -1, 1024)
        best = np.maximum(best, s.max(axis=2))
    thr = 5.0
    sp = SinglePulseSearch(threshold=thr, widths=widths, detrendlen=1024)
    got = sp(torch.from_numpy(z.astype(np.float32)).cuda(), dms=np.arange(R) * 1.0, dt=1e-3)
    gg = {(int(r), int(t) // 1024): float(s) for r, t, s in zip(got["row"], got["Sample"], got["Sigma"])}
    want = {(r, k): best[r, k] for r in range(R) for k in range(best.shape[1]) if best[r, k] >= thr}
    assert len(want) >= R
    for key in set(gg) | set(want):
        if key in gg and key in want:
            assert abs(gg[key] - want[key]) <= 1e-4 * max(1.0, abs(want[key])), (key, gg[key], want[key])
        else:
            s = gg.get(key, want.get(key))
            assert abs(s - thr) <= 1e-4 * thr, (key, s)
