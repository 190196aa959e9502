"""ORACLE (test infrastructure only; see oracle/__init__.py).

NumPy restatement of the reference's PSRFITS data path, working on the
arrays a test wrote (not on the product's FITS reader):
  unpack_4bit   formats/psrfits.py:37-50
  read_subint   formats/psrfits.py:67-107  ((data*scales)+offsets)*weights
  get_spectra   formats/psrfits.py:140-183 (concatenate, transpose, skip/trunc,
                flip the band when it ascends)
Pinned: tests/test_psrfits.py checks every function here against
tests/golden/golden_psrfits.npz, the outputs of the reference's own
formats/psrfits.py executed in the build container
(tests/golden/make_golden_psrfits.py): bit-exact for 4/8/16/32-bit data and
both band orders.  The restatement follows the reference lines above,
including numpy's float32 promotion of uint8/int16 data times float32
scales.  No PSRFITS file from a real backend ships with the reference, so
parity with such files is unpinned.
"""
import numpy as np


def unpack_4bit(data):
    first_piece = np.bitwise_and(15, data)
    second_piece = data >> 4
    return np.dstack([first_piece, second_piece]).flatten()


def read_subint(raw, nbits, nsblk, nchan, scales, offsets, weights, apply_weights=True,
                apply_scales=True, apply_offsets=True):
    """raw: the subint's DATA column as stored (uint8 bytes for nbits <= 8,
    '>i2' for 16, '>f4' for 32)."""
    if nbits == 4:
        data = unpack_4bit(np.asarray(raw, dtype=np.uint8))
    else:
        data = np.array(raw)
    o = offsets if apply_offsets else 0
    s = scales if apply_scales else 1
    w = weights if apply_weights else 1
    data = data.reshape((nsblk, nchan))
    return ((data * s) + o) * w


def get_spectra(subints, nsblk, freqs, need_flipband, startsamp, N):
    """subints: list of read_subint results ([nsblk, nchan] each) of the file
    from subint 0; returns (data [nchan, N], freqs) as get_spectra builds
    them before the Spectra constructor."""
    startsub = int(startsamp / nsblk)
    skip = startsamp - (startsub * nsblk)
    endsub = int((startsamp + N) / nsblk)
    trunc = ((endsub + 1) * nsblk) - (startsamp + N)
    data = [subints[i] if i < len(subints) else np.zeros_like(subints[0])
            for i in range(startsub, endsub + 1)]
    data = np.concatenate(data) if len(data) > 1 else np.array(data).squeeze()
    data = np.transpose(data)
    if trunc > 0:
        data = data[:, skip:-trunc]
    elif trunc == 0:
        data = data[:, skip:]
    if not need_flipband:
        data = data[::-1, :]
        freqs = freqs[::-1]
    return data, freqs
