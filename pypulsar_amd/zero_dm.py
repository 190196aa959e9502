"""Zero-DM filter on the GPU (drop-in for bin/zero_dm_filter.py:30-50).

Per spectrum (one time sample, all channels): subtract the channel mean.
Integer data (8/16-bit): the float64 mean is rounded half-to-even and cast to
the data type, and the subtraction wraps modulo 2**nbits -- exactly what the
reference's ``data - np.round(avg).astype(data.dtype)`` does.  float32 data:
float32 mean, float32 result.
"""
import numpy as np
import torch

from . import _lib
from ._lib import call, ptr, stream_ptr

_CODES = {torch.uint8: _lib.U8, torch.float32: _lib.F32}
_NP = {np.dtype(np.uint8): torch.uint8, np.dtype(np.float32): torch.float32}


def _code(t):
    if t.dtype == torch.uint8:
        return _lib.U8
    if t.dtype == torch.float32:
        return _lib.F32
    if t.dtype == torch.int16 and getattr(t, "_pdd_u16", False):
        return _lib.U16
    raise TypeError("zero-DM input must be uint8, uint16 or float32")


def zero_dm(block, layout="time", out=None):
    """Zero-DM filter a block on the device.

    block: [nspec, nchan] ('time' layout, filterbank order) or [nchan, nspec]
    ('chan' layout, Spectra order) device tensor of uint8 / float32, or a numpy
    array of uint8 / uint16 / float32 (uploaded; the result comes back as a
    numpy array of the same dtype).  ``out`` may be ``block`` (in place)."""
    _lib.require_gpu()
    host = isinstance(block, np.ndarray)
    code16 = False
    if host:
        a = np.ascontiguousarray(block)
        if a.dtype == np.uint16:
            code16 = True
            t = torch.from_numpy(a.view(np.int16)).cuda()
        elif a.dtype in (np.uint8, np.float32):
            t = torch.from_numpy(a).cuda()
        else:
            raise TypeError("zero-DM input must be uint8, uint16 or float32")
    else:
        t = block
    code = _lib.U16 if code16 else _code(t)
    if t.stride(1) != 1:
        t = t.contiguous()
    if layout == "time":
        nspec, nchan = t.shape
        lay = _lib.LAYOUT_TIME_MAJOR
    elif layout == "chan":
        nchan, nspec = t.shape
        lay = _lib.LAYOUT_CHAN_MAJOR
    else:
        raise ValueError("layout must be 'time' or 'chan'")
    if out is None:
        out = torch.empty_like(t)
    call("pdd_zero_dm", ptr(t), code, nspec, nchan, t.stride(0), lay, ptr(out), out.stride(0),
         stream_ptr())
    if host:
        r = out.cpu().numpy()
        return r.view(np.uint16) if code16 else r
    return out
