"""SIGPROC header codec and filterbank reader (host side; drop-in for
formats/filterbank.py:19-157 and PRESTO's sigproc header functions).
PRESTO is absent, so header parity with PRESTO is unpinned: the codec is
checked on hand-built bytes of the public SIGPROC format and by round trips."""
import os
import struct
import warnings

import numpy as np
import pytest

from pypulsar_amd.formats import filterbank as fbm
from pypulsar_amd.formats import sigproc


def _s(x):
    b = x.encode()
    return struct.pack("<i", len(b)) + b


def test_hand_built_header(tmp_path):
    raw = (_s("HEADER_START") + _s("nchans") + struct.pack("<i", 4) + _s("nbits") +
           struct.pack("<i", 8) + _s("tsamp") + struct.pack("<d", 6.4e-5) + _s("fch1") +
           struct.pack("<d", 1500.0) + _s("foff") + struct.pack("<d", -1.5) + _s("source_name") +
           _s("B0000+00") + _s("signed") + struct.pack("<b", 0) + _s("HEADER_END"))
    data = np.arange(24, dtype=np.uint8).reshape(6, 4)
    fn = tmp_path / "x.fil"
    fn.write_bytes(raw + data.tobytes())
    fb = fbm.filterbank(str(fn))
    assert fb.header_size == len(raw)
    assert fb.header_params[0] == "HEADER_START" and fb.header_params[-1] == "HEADER_END"
    assert fb.nchans == 4 and fb.nbits == 8 and fb.tsamp == 6.4e-5 and fb.source_name == "B0000+00"
    assert fb.number_of_samples == 6 and fb.dtype == "uint8"
    np.testing.assert_array_equal(fb.frequencies, 1500.0 - 1.5 * np.arange(4))
    assert fb.is_hifreq_first
    fb.seek_to_sample(2)
    np.testing.assert_array_equal(fb.read_sample(), data[2])
    np.testing.assert_array_equal(fb.read_Nsamples(2).reshape(2, 4), data[3:5])
    np.testing.assert_array_equal(fb.read_all_samples().reshape(6, 4), data)
    fb.close()


@pytest.mark.parametrize("nbits,dtype", [(8, np.uint8), (16, np.uint16), (32, np.float32)])
def test_round_trip(tmp_path, nbits, dtype):
    params, hdr = sigproc.make_header(32, nbits, 81.92e-6, 1400.0, 0.5, source_name="J1234")
    x = (np.random.default_rng(nbits).random((50, 32)) * 200).astype(dtype)
    fn = str(tmp_path / "r.fil")
    fbm.write_filterbank(fn, params, hdr, x)
    fb = fbm.filterbank(fn)
    assert fb.header_params == params
    for k in params:
        assert fb.header[k] == hdr[k]
    assert fb.number_of_samples == 50 and not fb.is_hifreq_first
    buf = np.empty((20, 32), dtype=dtype)
    assert fb.read_block_into(40, buf) == 10
    np.testing.assert_array_equal(buf[:10], x[40:])
    # a non-contiguous or mis-shaped destination is refused, not filled
    # through a temporary copy
    wide = np.zeros((20, 64), dtype=dtype)
    with pytest.raises(ValueError):
        fb.read_block_into(0, wide[:, ::2])
    with pytest.raises(ValueError):
        fb.read_block_into(0, np.zeros((20, 16), dtype=dtype))
    with pytest.raises(ValueError):
        fb.read_block_into(0, np.zeros((20, 32), dtype=np.int64))
    assert not wide.any()
    # re-written header bytes are identical (zero_dm_filter.py:21-27 path)
    with open(fn, "rb") as f:
        head = f.read(fb.header_size)
    out = tmp_path / "h.bin"
    with open(out, "wb") as f:
        sigproc.write_header(f, fb.header_params, fb.header)
    assert out.read_bytes() == head


def test_errors(tmp_path):
    with pytest.raises(ValueError):
        fbm.filterbank(str(tmp_path / "missing.fil"))
    bad = tmp_path / "bad.fil"
    bad.write_bytes(_s("HEADER_START") + _s("bogus_key") + b"\0" * 16)
    with pytest.raises(ValueError):
        fbm.filterbank(str(bad))
    params, hdr = sigproc.make_header(3, 8, 1e-3, 100.0, -1.0)
    fn = str(tmp_path / "odd.fil")
    fbm.write_filterbank(fn, params, hdr, np.zeros(10, np.uint8))  # 10 bytes: not 3 x n
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        fb = fbm.filterbank(fn)
    assert fb.number_of_samples == 3 and any("integer number" in str(x.message) for x in w)
    with pytest.raises(AttributeError):
        fb.not_a_header_key  # noqa: B018
