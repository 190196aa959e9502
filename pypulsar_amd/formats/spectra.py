"""Device-resident ``Spectra``: the drop-in for pypulsar's formats/spectra.py.

Same constructor, attributes, method names, argument meanings and assertion
behaviour as the reference class (formats/spectra.py:8-351).  The data live in
HBM as float32 ``[numchans, numspectra]`` (a strided view of a device buffer so
``trim`` never copies); every hot-path method runs a hand-written HIP kernel
of libpdd.so through the C ABI (include/pdd.h).  There is no CPU fallback:
without a GPU or without libpdd.so the methods raise.

Documented differences from the reference:
  * float32 on device instead of float64 (parity: integer-valued data and
    integer pads are bit-exact; otherwise 1e-5 relative);
  * ``.data`` is a float64 host copy (one device->host transfer per access)
    that WRITES THROUGH: ``s.data[...] = v``, ``chan = s.get_chan(i);
    chan[:] = v`` and in-place arithmetic on those arrays or their slices
    upload the modified array back to the device, like the reference's views
    into its own ndarray (formats/spectra.py:42-52); a view taken before the
    Spectra was modified again (dedisperse, trim, ...) raises instead of
    overwriting the newer data.
"""
import copy
import weakref

import numpy as np
import torch

from .. import _lib
from .._lib import call, ptr, stream_ptr
from .. import delays as _delays


def _np_dtype_code(dt):
    if dt == np.uint8:
        return _lib.U8
    if dt == np.uint16:
        return _lib.U16
    if dt == np.float32:
        return _lib.F32
    return None


def _torch_dtype_code(dt):
    return {torch.uint8: _lib.U8, torch.float32: _lib.F32}.get(dt)


def upload_f32(data):
    """Copy a [C, N] array (numpy, any order/dtype, or torch) to a new
    contiguous float32 device tensor through libpdd (corner turn for the
    transposed filterbank layout, conversion for u8/u16/f32).  Also returns
    the raw 8-bit [C, N] device copy when the input is uint8 (for the 8-bit
    sweep kernel), else None."""
    _lib.require_gpu()
    dev = torch.device("cuda")
    if isinstance(data, torch.Tensor):
        t = data
        if t.dim() != 2:
            raise ValueError("data must be 2-D")
        C, N = t.shape
        if t.dtype not in (torch.uint8, torch.float32):
            t = t.to(torch.float32)
        t = t.to(dev)
        code = _torch_dtype_code(t.dtype)
        out = torch.empty((C, N), dtype=torch.float32, device=dev)
        raw8 = None
        if t.stride(1) == 1:
            call("pdd_convert_f32", ptr(t), code, C, N, t.stride(0), ptr(out), N, stream_ptr())
            if t.dtype == torch.uint8:
                raw8 = t.contiguous().clone()
        elif t.stride(0) == 1:  # transposed [N, C] storage
            call("pdd_corner_turn", ptr(t), code, N, C, t.stride(1), ptr(out), _lib.F32, N,
                 stream_ptr())
            if t.dtype == torch.uint8:
                raw8 = t.contiguous()
        else:
            tc = t.contiguous()
            call("pdd_convert_f32", ptr(tc), code, C, N, N, ptr(out), N, stream_ptr())
            if t.dtype == torch.uint8:
                raw8 = tc.clone()
        return out, raw8

    a = np.asarray(data)
    if a.ndim != 2:
        raise ValueError("data must be 2-D")
    C, N = a.shape
    code = _np_dtype_code(a.dtype)
    if code is None:
        a = a.astype(np.float32)
        code = _lib.F32
    out = torch.empty((C, N), dtype=torch.float32, device=dev)
    raw8 = None
    if C == 0 or N == 0:
        return out, None
    if a.T.flags.c_contiguous and not a.flags.c_contiguous:
        # the layout filterbank.get_spectra hands over: data.T of an [N, C] block
        src = torch.from_numpy(np.ascontiguousarray(a.T)).to(dev, non_blocking=False)
        call("pdd_corner_turn", ptr(src), code, N, C, C, ptr(out), _lib.F32, N, stream_ptr())
        if code == _lib.U8:
            raw8 = torch.empty((C, N), dtype=torch.uint8, device=dev)
            call("pdd_corner_turn", ptr(src), code, N, C, C, ptr(raw8), _lib.U8, N, stream_ptr())
    else:
        src = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        call("pdd_convert_f32", ptr(src), code, C, N, N, ptr(out), N, stream_ptr())
        if code == _lib.U8:
            raw8 = src
    return out, raw8


def _pad_args(x, padval):
    """(pad_mode, padvals device tensor or None) for a [C, N] float32 view,
    the semantics of spectra.py:81-94."""
    C = x.shape[0]
    if isinstance(padval, str):
        if padval == "rotate":
            return _lib.PAD_ROTATE, None
        if padval in ("mean", "median"):
            stat = _lib.STAT_MEAN if padval == "mean" else _lib.STAT_MEDIAN
            pv = torch.empty(C, dtype=torch.float32, device=x.device)
            call("pdd_channel_stats", ptr(x), C, x.shape[1], x.stride(0), stat, ptr(pv),
                 stream_ptr())
            return _lib.PAD_VALUE, pv
        raise ValueError("padval must be a number, 'mean', 'median' or 'rotate'")
    pv = torch.full((C,), float(padval), dtype=torch.float32, device=x.device)
    return _lib.PAD_VALUE, pv


class HostView(np.ndarray):
    """float64 host copy of a Spectra's device data whose writes go back to
    the device: ``__setitem__`` and in-place ufuncs on it -- or on any slice
    of it (they share its memory) -- upload the whole copy.  Reference idiom
    kept: ``chan = s.get_chan(i); chan[:] = v`` changes channel i
    (formats/spectra.py:48-52: get_chan returns a view into self.data).
    While the device data is unchanged, ``s.data`` / ``get_chan`` /
    ``get_spectrum`` hand out views of ONE host copy (as the reference's
    views share ``self.data``), so writes through two open views both land;
    a view taken before a device-side change raises on write."""

    def __array_finalize__(self, obj):
        self._root = getattr(obj, "_root", None)

    def _push(self):
        root = self._root
        if root is None:
            return
        s, version = root._owner
        if s._version != version:
            raise RuntimeError("Spectra was modified after this view of its data was taken; "
                               "take a new view (s.data / get_chan / get_spectrum)")
        s._upload_host(np.asarray(root).view(np.ndarray))
        root._owner = (s, s._version)

    def __setitem__(self, key, value):
        super(HostView, self).__setitem__(key, value)
        self._push()

    # in-place ndarray methods that bypass __setitem__ and ufuncs
    def fill(self, value):
        np.ndarray.fill(self, value)
        self._push()

    def put(self, *args, **kwargs):
        np.ndarray.put(self, *args, **kwargs)
        self._push()

    def sort(self, *args, **kwargs):
        np.ndarray.sort(self, *args, **kwargs)
        self._push()

    def partition(self, *args, **kwargs):
        np.ndarray.partition(self, *args, **kwargs)
        self._push()

    def __array_ufunc__(self, ufunc, method, *inputs, **kwargs):
        args = [np.asarray(a).view(np.ndarray) if isinstance(a, HostView) else a for a in inputs]
        outs = kwargs.get("out")
        if outs:
            kwargs["out"] = tuple(np.asarray(o).view(np.ndarray) if isinstance(o, HostView) else o
                                  for o in outs)
        res = getattr(ufunc, method)(*args, **kwargs)
        if outs:
            for o in outs:
                if isinstance(o, HostView):
                    o._push()
            return outs[0] if len(outs) == 1 else outs
        return res


def _bins_dev(bins, device):
    return torch.from_numpy(_delays.to_int32(bins)).to(device)


class Spectra(object):
    """A [numchans, numspectra] block of filterbank data on the GPU."""

    def __init__(self, freqs, dt, data, starttime=0, dm=0):
        self.numchans, self.numspectra = data.shape
        assert len(freqs) == self.numchans
        self.freqs = freqs
        self._x, self._raw8 = upload_f32(data)
        self._version = 0
        self.dt = dt
        self.starttime = starttime
        self.dm = 0  # the reference ignores the dm argument (spectra.py:37)

    @classmethod
    def _from_device(cls, freqs, dt, x, starttime=0):
        """Adopt a float32 [numchans, numspectra] device tensor produced by a
        reader kernel (no copy; the readers' own data, so the reference's
        always-copy constructor semantics are kept)."""
        assert x.dtype == torch.float32 and x.dim() == 2 and x.stride(1) == 1
        self = cls.__new__(cls)
        self.numchans, self.numspectra = x.shape
        assert len(freqs) == self.numchans
        self.freqs = freqs
        self._x, self._raw8 = x, None
        self._version = 0
        self.dt = dt
        self.starttime = starttime
        self.dm = 0
        return self

    # ------------------------------------------------------------ data access
    @property
    def device_data(self):
        """The float32 [numchans, numspectra] device view (no copy)."""
        return self._x

    @property
    def data(self):
        """float64 host copy of the data that writes through to the device
        (HostView).  One copy per device version, shared by every view taken
        while the device data is unchanged (weakly cached)."""
        ref = getattr(self, "_host", None)
        if ref is not None and ref[0] == self._version:
            v = ref[1]()
            if v is not None:
                return v
        v = self._x.to(torch.float64).cpu().numpy().view(HostView)
        v._root = v
        v._owner = (self, self._version)
        self._host = (self._version, weakref.ref(v))
        return v

    @data.setter
    def data(self, value):
        self._x, self._raw8 = upload_f32(value)
        self.numchans, self.numspectra = self._x.shape
        self._version = getattr(self, "_version", 0) + 1

    def _upload_host(self, arr):
        """Write a full [numchans, numspectra] host array back (HostView).
        The shared host copy is rounded in place to the float32 values the
        device now holds, so it stays equal to the device and the version
        (and the copy's validity) is unchanged."""
        assert arr.shape == tuple(self._x.shape)
        f32 = np.ascontiguousarray(arr, dtype=np.float32)
        self._x.copy_(torch.from_numpy(f32))
        arr[...] = f32
        self._raw8 = None

    def _set(self, x):
        self._x = x
        self._raw8 = None
        self._version = getattr(self, "_version", 0) + 1

    def __str__(self):
        return str(np.asarray(self.data))

    def __getitem__(self, key):
        return self.data[key]

    def __setitem__(self, key, value):
        if not isinstance(value, torch.Tensor):
            value = torch.as_tensor(np.asarray(value, dtype=np.float32))
        self._x[key] = value.to(device=self._x.device, dtype=torch.float32)
        self._raw8 = None
        self._version = getattr(self, "_version", 0) + 1

    def get_chan(self, channum):
        return self.data[channum, :]

    def get_spectrum(self, specnum):
        return self.data[:, specnum]

    def __deepcopy__(self, memo):
        other = copy.copy(self)
        other._version = 0
        other._host = None  # never share the original's host copy
        other._x = self._x.clone()
        other._raw8 = None if self._raw8 is None else self._raw8.clone()
        other.freqs = copy.deepcopy(self.freqs, memo)
        return other

    # ------------------------------------------------------------ hot path
    def shift_channels(self, bins, padval=0):
        """Shift each channel left by bins[c] and pad (spectra.py:54-94)."""
        assert self.numchans == len(bins)
        x = self._x
        C, N = x.shape
        if C == 0 or N == 0:
            return
        mode, pv = _pad_args(x, padval)
        out = torch.empty((C, N), dtype=torch.float32, device=x.device)
        b = _bins_dev(bins, x.device)
        call("pdd_shift_pad", ptr(x), C, N, x.stride(0), ptr(b), mode, ptr(pv), ptr(out), N, N,
             stream_ptr())
        self._set(out)

    def subband(self, nsub, subdm=None, padval=0):
        """Shift within subbands at subdm and sum them (spectra.py:96-138).
        ``self.dm`` is not changed (as in the reference)."""
        assert (self.numchans % nsub) == 0
        assert (subdm is None) or (subdm >= 0)
        freqs = np.asarray(self.freqs, dtype=np.float64)
        _, _, ctr = _delays.subband_layout(freqs, nsub)
        x = self._x
        C, N = x.shape
        out = torch.empty((nsub, N), dtype=torch.float32, device=x.device)
        if N > 0:
            if subdm is not None:
                bins = _delays.subband_bins(subdm, freqs, self.dt, nsub, cur_dm=self.dm)
                b = _bins_dev(bins, x.device)
                mode, pv = _pad_args(x, padval)
            else:
                b, mode, pv = None, _lib.PAD_VALUE, None
            call("pdd_shift_group_sum", ptr(x), C, N, x.stride(0), ptr(b), mode, ptr(pv), nsub,
                 ptr(out), N, N, stream_ptr())
        self._set(out)
        self.freqs = ctr
        self.numchans = nsub

    def dedisperse(self, dm=0, padval=0, trim=False):
        """Shift channels by the delays of ``dm`` (spectra.py:229-260)."""
        assert dm >= 0
        bins = _delays.dedisperse_bins(dm, self.freqs, self.dt, cur_dm=self.dm)
        self.shift_channels(bins, padval)
        self.dm = dm
        if trim:
            ntrim = int(max(bins))
            if ntrim > 0:
                self._set(self._x[:, :max(0, self._x.shape[1] - ntrim)])
                self.numspectra -= ntrim

    def trim(self, bins=0):
        """Drop ``bins`` samples from the end (or -bins from the start),
        spectra.py:305-327 -- including the reference's numspectra arithmetic
        for negative bins."""
        assert bins < self.numspectra
        if bins == 0:
            return
        elif bins > 0:
            self._set(self._x[:, :-bins])
            self.numspectra = self.numspectra - bins
        elif bins < 0:
            self._set(self._x[:, bins:])
            self.numspectra = self.numspectra - bins
            self.starttime = self.starttime + bins * self.dt

    def downsample(self, factor=1, trim=True):
        """Co-add ``factor`` adjacent samples (spectra.py:329-351)."""
        assert trim or not (self.numspectra % factor)
        new_num_spectra = self.numspectra // factor
        self.trim(self.numspectra % factor)
        x = self._x
        C, N = x.shape
        out = torch.empty((C, new_num_spectra), dtype=torch.float32, device=x.device)
        if C and new_num_spectra:
            call("pdd_downsample", ptr(x), C, N, x.stride(0), factor, ptr(out), new_num_spectra,
                 stream_ptr())
        self._set(out)
        self.numspectra = new_num_spectra
        self.dt = self.dt * factor

    # ------------------------------------------------------------ post-chain
    # waterfaller.py:120-127 continues with scaled() and smooth(); masked() is
    # its rfifind mask step (waterfaller.py:92-99).  All return / modify the
    # device data like the reference (copies vs in place as documented there).
    def _stat(self, x, stat):
        v = torch.empty(x.shape[0], dtype=torch.float32, device=x.device)
        call("pdd_channel_stats", ptr(x), x.shape[0], x.shape[1], x.stride(0), stat, ptr(v),
             stream_ptr())
        return v

    def _global(self, x):
        g = torch.empty(4, dtype=torch.float32, device=x.device)  # mean, std, min, max
        call("pdd_global_stats", ptr(x), x.shape[0], x.shape[1], x.stride(0), ptr(g), stream_ptr())
        return g

    def _scale(self, x, sub, sub_inc, div, div_inc):
        C, N = x.shape
        out = torch.empty((C, N), dtype=torch.float32, device=x.device)
        call("pdd_scale_rows", ptr(x), C, N, x.stride(0), ptr(sub), sub_inc, ptr(div), div_inc,
             ptr(out), N, stream_ptr())
        return out

    def scaled(self, indep=False):
        """Copy with every channel minus its median, divided by the global
        std (indep=False) or the channel's std (spectra.py:140-163)."""
        other = copy.deepcopy(self)
        x = other._x
        if x.numel() == 0:
            return other
        med = self._stat(x, _lib.STAT_MEDIAN)
        if indep:
            std, inc = self._stat(x, _lib.STAT_STD), 1
        else:
            std, inc = self._global(x)[1:2], 0
        other._set(self._scale(x, med, 1, std, inc))
        return other

    def scaled2(self, indep=False):
        """Copy with every channel minus its minimum, divided by the global
        maximum (indep=False) or the channel's maximum (spectra.py:165-188)."""
        other = copy.deepcopy(self)
        x = other._x
        if x.numel() == 0:
            return other
        mn = self._stat(x, _lib.STAT_MIN)
        if indep:
            mx, inc = self._stat(x, _lib.STAT_MAX), 1
        else:
            mx, inc = self._global(x)[3:4], 0
        other._set(self._scale(x, mn, 1, mx, inc))
        return other

    def masked(self, mask, maskval="median-mid80"):
        """Copy with masked entries replaced by ``maskval`` per channel: a
        number, 'mean', 'median' or 'median-mid80' (spectra.py:190-227).
        'median-mid80' is the median of the middle 80% of the sorted channel,
        which equals the channel median, except when round(0.1 N) == 0, where
        the reference's slice is empty and its value is NaN."""
        mask = np.asarray(mask)
        assert (self.numchans, self.numspectra) == mask.shape
        other = copy.deepcopy(self)
        x = other._x
        C, N = x.shape
        if C == 0 or N == 0:
            return other
        if maskval == "mean":
            vals = self._stat(x, _lib.STAT_MEAN)
        elif maskval in ("median", "median-mid80"):
            if maskval == "median-mid80" and int(np.round(0.1 * self.numspectra)) == 0:
                vals = torch.full((C,), float("nan"), dtype=torch.float32, device=x.device)
            else:
                vals = self._stat(x, _lib.STAT_MEDIAN)
        else:
            vals = torch.full((C,), float(maskval), dtype=torch.float32, device=x.device)
        m = torch.from_numpy(np.ascontiguousarray(mask, dtype=np.uint8)).to(x.device)
        out = torch.empty((C, N), dtype=torch.float32, device=x.device)
        call("pdd_masked_fill", ptr(x), C, N, x.stride(0), ptr(m), N, ptr(vals), ptr(out), N,
             stream_ptr())
        other._set(out)
        return other

    def smooth(self, width=1, padval=0):
        """In place: convolve every channel with a boxcar of ``width`` samples
        and height 1/sqrt(width); overlap values from ``padval`` (a number,
        'mean', 'median' or 'wrap') (spectra.py:262-303)."""
        if width <= 1:
            return
        x = self._x
        C, N = x.shape
        if C == 0 or N == 0:
            return
        if padval == "wrap":
            mode, pv = _lib.PAD_ROTATE, None
        elif padval in ("mean", "median"):
            mode, pv = _lib.PAD_VALUE, self._stat(x, _lib.STAT_MEAN if padval == "mean"
                                                   else _lib.STAT_MEDIAN)
        else:
            mode = _lib.PAD_VALUE
            pv = torch.full((C,), float(padval), dtype=torch.float32, device=x.device)
        out = torch.empty((C, N), dtype=torch.float32, device=x.device)
        call("pdd_smooth", ptr(x), C, N, x.stride(0), int(width), mode, ptr(pv), ptr(out), N,
             stream_ptr())
        self._set(out)

    # ------------------------------------------------------------ fused extras
    def sum_channels(self):
        """Device float32 [numspectra] series = data.sum(axis=0)
        (bin/waterfaller.py:140), float64 accumulation in the kernel."""
        x = self._x
        C, N = x.shape
        out = torch.empty((1, N), dtype=torch.float32, device=x.device)
        if N:
            call("pdd_shift_group_sum", ptr(x), C, N, x.stride(0), None, _lib.PAD_VALUE, None, 1,
                 ptr(out), N, N, stream_ptr())
        return out[0]

    def dedispersed_series(self, dm, padval=0, trim=True):
        """Fused dedisperse(dm, padval, trim) + channel sum WITHOUT modifying
        this Spectra: one pass over the data (pdd_shift_group_sum, nsub=1)."""
        assert dm >= 0
        bins = _delays.dedisperse_bins(dm, self.freqs, self.dt, cur_dm=self.dm)
        x = self._x
        C, N = x.shape
        ntrim = int(max(bins)) if trim else 0
        n_out = N - ntrim if ntrim > 0 else N
        n_out = max(0, n_out)
        out = torch.empty((1, max(1, n_out)), dtype=torch.float32, device=x.device)
        if n_out:
            mode, pv = _pad_args(x, padval)
            b = _bins_dev(bins, x.device)
            call("pdd_shift_group_sum", ptr(x), C, N, x.stride(0), ptr(b), mode, ptr(pv), 1,
                 ptr(out), n_out, n_out, stream_ptr())
        return out[0, :n_out]

    def sweep(self, dms, padval=0, trim=True, plane=None):
        """Batched DM-trial sweep of this Spectra (new executor): returns
        the float32 device plane [len(dms), n_out], row d = the dedispersed
        series of ``dedisperse(dms[d], padval, trim)``, truncated to the
        common length (trim=True) or full length (trim=False)."""
        from ..sweep import DMSweep
        sw = DMSweep(dms, self.freqs, self.dt, cur_dm=self.dm,
                     dtype="u8" if (self._raw8 is not None) else "f32")
        return sw(self, padval=padval, trim=trim, out=plane)
