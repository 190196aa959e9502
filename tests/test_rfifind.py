"""rfifind .mask reader (pypulsar_amd.formats.rfifind) on the CPU: byte
layout, write -> read round trips and get_mask (bin/waterfaller.py:28-48).
Parity with PRESTO's own reader is unpinned (PRESTO is absent and the
reference ships no mask file)."""
import struct

import numpy as np
import pytest

from pypulsar_amd.formats import rfifind as rf


def _per_int(nchan, nint, seed):
    rng = np.random.default_rng(seed)
    per = []
    for i in range(nint):
        k = [0, nchan, 1, 5][i % 4] if i < 4 else int(rng.integers(0, nchan // 2))
        per.append(np.sort(rng.choice(nchan, size=k, replace=False)).astype(np.int32))
    return per


def test_layout_by_hand(tmp_path):
    fn = str(tmp_path / "a_rfifind.mask")
    hdr = struct.pack("<6d3i", 10.0, 4.0, 55000.5, 2.0, 1200.0, 0.5, 8, 3, 100)
    body = struct.pack("<i2i", 2, 1, 6) + struct.pack("<i", 0)
    body += struct.pack("<3i", 2, 8, 0) + struct.pack("<2i", 3, 4)
    open(fn, "wb").write(hdr + body)
    m = rf.rfifind(fn)
    assert (m.nchan, m.nint, m.ptsperint) == (8, 3, 100)
    assert m.MJD == 55000.5 and m.dtint == 2.0 and m.basename == str(tmp_path / "a")
    np.testing.assert_array_equal(m.freqs, 1200.0 + 0.5 * np.arange(8))
    assert m.mask_zap_chans == {1, 6} and len(m.mask_zap_ints) == 0
    assert [list(z) for z in m.mask_zap_chans_per_int] == [[3, 4], list(range(8)), []]


def test_truncated(tmp_path):
    fn = str(tmp_path / "t.mask")
    rf.write_mask(fn, 16, 64, _per_int(16, 6, 1))
    open(fn, "ab").close()
    data = open(fn, "rb").read()
    open(fn, "wb").write(data[:-4])
    with pytest.raises(ValueError):
        rf.rfifind(fn)


@pytest.mark.parametrize("start,N", [(0, 1000), (37, 777), (640, 64), (1000, 1)])
def test_round_trip_and_get_mask(tmp_path, start, N):
    nchan, nint, ppi = 32, 20, 64
    per = _per_int(nchan, nint, 4)
    fn = str(tmp_path / "x.mask")
    rf.write_mask(fn, nchan, ppi, per, zap_chans=[3, 7], zap_ints=[2])
    m = rf.rfifind(fn)
    assert len(m.mask_zap_chans_per_int) == nint
    for a, b in zip(m.mask_zap_chans_per_int, per):
        np.testing.assert_array_equal(np.sort(a), b)
    assert list(m.mask_zap_ints) == [2]
    mask = rf.get_mask(m, start, N)
    assert mask.shape == (nchan, N) and mask.dtype == bool
    for j in range(N):  # the reference's per-sample definition
        want = np.zeros(nchan, bool)
        want[per[(start + j) // ppi]] = True
        np.testing.assert_array_equal(mask[:, j], want)


def test_get_mask_past_the_end(tmp_path):
    fn = str(tmp_path / "x.mask")
    rf.write_mask(fn, 8, 10, _per_int(8, 3, 2))
    with pytest.raises(IndexError):
        rf.get_mask(rf.rfifind(fn), 25, 10)
