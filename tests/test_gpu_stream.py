"""Streaming pipeline (pypulsar_amd.stream; BASELINE config 5) on the GPU:
the fused zero-DM + downsample prologue against the oracle, and the
concatenated per-block planes against the one-shot plane (bit-identical:
same kernels, every column sees all of its inputs)."""
import numpy as np
import pytest

from conftest import band, rel_err, u8_data
from oracle import spectra_oracle as orc

pytestmark = pytest.mark.gpu
DT = 64e-6


@pytest.mark.parametrize("dtype", [np.uint8, np.float32])
@pytest.mark.parametrize("factor", [1, 2, 8])
@pytest.mark.parametrize("zdm", [0, 1])
def test_zdm_downsample(gpu, dtype, factor, zdm):
    import torch
    from pypulsar_amd import _lib
    from pypulsar_amd._lib import call, ptr, stream_ptr
    nspec, C = 1000 + factor - 1, 70
    x = (u8_data(nspec, C, 5) if dtype == np.uint8
         else np.random.default_rng(5).normal(0, 3, (nspec, C)).astype(np.float32))
    xd = torch.from_numpy(x).cuda()
    out = torch.zeros((C, nspec // factor), dtype=torch.float32, device="cuda")
    code = _lib.U8 if dtype == np.uint8 else _lib.F32
    call("pdd_zdm_downsample", ptr(xd), code, nspec, C, C, factor, zdm, ptr(out), out.stride(0),
         stream_ptr())
    want = orc.zdm_downsample(x, factor, bool(zdm))
    got = out.cpu().numpy()
    if dtype == np.uint8 and not zdm:
        np.testing.assert_array_equal(got, want)
    else:
        assert rel_err(got, want) <= 1e-5


@pytest.mark.parametrize("mode,factor", [("int", 1), ("int", 2), ("wrap", 2), ("wrap", 4),
                                         ("none", 4)])
def test_zdm_int_downsample(gpu, mode, factor):
    """Integer prologue of the exact 16-bit stream path, bit-exact against the
    oracle (incl. the reference's uint8 wrap, zero_dm_filter.py:30-39)."""
    import torch
    from pypulsar_amd import _lib
    from pypulsar_amd.stream import prologue
    nspec, C = 1000 + factor - 1, 96
    x = u8_data(nspec, C, 7)
    x[:5] = 255   # extreme spectra: differences at +-255
    x[5:9, :48] = 0
    x[9] = np.arange(C) % 2 * 255  # mean 127.5: the half-to-even tie
    xd = torch.from_numpy(x).cuda()
    img = torch.full((C, nspec // factor + 3), -1, dtype=torch.int16, device="cuda")
    off = 255 * factor if mode == "int" else 0
    prologue(xd, nspec, C, factor, mode, img, off)
    got = img.cpu().numpy().astype(np.int64) & 0xffff
    want = orc.zdm_int_downsample(x, factor, mode) + off
    np.testing.assert_array_equal(got[:, :nspec // factor], want)
    assert (got[:, nspec // factor:] == 0xffff).all()  # nothing past n_out written


def test_sweep_u16_with_bias(gpu):
    """16-bit sweep input (values <= 1023, the 64-channel flush) and the
    epilogue bias: bit-exact against the oracle plane."""
    import torch
    from pypulsar_amd.sweep import DMSweep
    C, N = 200, 6000
    freqs = band(C)
    rng = np.random.default_rng(11)
    x = rng.integers(0, 1024, (C, N)).astype(np.int16)
    x[:, :50] = 1023  # carries would show at the maximum
    dms = np.linspace(0.0, 150.0, 50)
    sw = DMSweep(dms, freqs, DT, dtype="u16")
    got = sw(torch.from_numpy(x).cuda(), out_bias=-1000.0 * C).cpu().numpy()
    want = orc.sweep_plane(x.astype(np.float64), orc.sweep_table(dms, freqs, DT)) - 1000.0 * C
    np.testing.assert_array_equal(got, want)
    sw.close()


@pytest.mark.parametrize("nchunks,last,zdm", [(3, 4096, "float"), (4, 1000, "float"),
                                             (3, 4096, "int"), (4, 1000, "int"),
                                             (3, 1000, "wrap")])
def test_stream_equals_one_shot(gpu, nchunks, last, zdm):
    import torch
    from pypulsar_amd.stream import StreamingSweep
    from pypulsar_amd.sweep import DMSweep
    C, block, ds = 96, 4096, 2
    freqs = band(C)
    dms = np.linspace(0.0, 200.0, 40)  # max delay 2900 input spectra < block
    N = block * (nchunks - 1) + last
    x = u8_data(N, C, 17)  # [time, chan], file order
    st = StreamingSweep(dms, freqs, DT, block=block, downsamp=ds, zero_dm=zdm)
    assert st.exact == (zdm != "float")
    chunks = [torch.from_numpy(x[i:i + block]).pin_memory() for i in range(0, N, block)]
    parts = [(t0, p.cpu().numpy()) for t0, p in st(chunks)]
    torch.cuda.synchronize()
    got = np.concatenate([p for _, p in parts], axis=1)
    assert [t0 for t0, _ in parts] == list(np.cumsum([0] + [p.shape[1] for _, p in parts[:-1]]))
    if zdm != "float":
        # exact integer path: the oracle composition bit for bit
        ref = orc.sweep_plane(orc.zdm_int_downsample(x, ds, zdm).astype(np.float64),
                              orc.sweep_table(dms, freqs, DT * ds))
        assert got.shape == ref.shape
        np.testing.assert_array_equal(got, ref)
        st.close()
        return
    # one-shot on the device: same prologue + sweep over the whole stream
    from pypulsar_amd import _lib
    from pypulsar_amd._lib import call, ptr, stream_ptr
    xd = torch.from_numpy(x).cuda()
    f32 = torch.empty((C, N // ds), dtype=torch.float32, device="cuda")
    call("pdd_zdm_downsample", ptr(xd), _lib.U8, N, C, C, ds, 1, ptr(f32), f32.stride(0),
         stream_ptr())
    want = DMSweep(dms, freqs, DT * ds)(f32).cpu().numpy()
    assert got.shape == want.shape
    np.testing.assert_array_equal(got, want)
    # and the oracle composition (float tolerance: zero-DM makes data fractional)
    ref = orc.sweep_plane(orc.zdm_downsample(x, ds), orc.sweep_table(dms, freqs, DT * ds))
    assert rel_err(got, ref) <= 1e-5
    st.close()


@pytest.mark.parametrize("zdm", ["int", "float"])
def test_stream_restart_by_block_index(gpu, zdm):
    """A stream resumed at block k (chunks k.., start_block=k) yields exactly
    the (t0, plane) pairs of blocks k.. of the uninterrupted run."""
    import torch
    from pypulsar_amd.stream import StreamingSweep
    C, block, ds = 96, 4096, 2
    freqs = band(C)
    dms = np.linspace(0.0, 200.0, 40)
    N = block * 4 + 1000
    x = u8_data(N, C, 23)
    st = StreamingSweep(dms, freqs, DT, block=block, downsamp=ds, zero_dm=zdm)
    chunks = [torch.from_numpy(x[i:i + block]).pin_memory() for i in range(0, N, block)]
    full = [(t0, p.cpu().numpy()) for t0, p in st(chunks)]
    for k in (1, 3):
        part = [(t0, p.cpu().numpy()) for t0, p in st(chunks[k:], start_block=k)]
        assert len(part) == len(full) - k
        for (ta, pa), (tb, pb) in zip(part, full[k:]):
            assert ta == tb
            np.testing.assert_array_equal(pa, pb)
    st.close()
