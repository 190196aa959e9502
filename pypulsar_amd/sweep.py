"""Batched DM-trial sweep and the DDplan executor (new; no reference executor).

Semantics, per DM trial d:
    row_d = Spectra.dedisperse(dms[d], padval, trim).data.sum(axis=0)
(formats/spectra.py:229-260 + bin/waterfaller.py:140).  The plane holds all
rows with a common length: N - max(0, max bins) when trim=True (every row is
then the prefix of the reference row), N when trim=False.

The delay table is built ONCE per (grid, channel frequencies, dt) on the host
in float64 (bit-exact) and the device plan (pdd_sweep_plan) keeps it in HBM.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import call, ptr, stream_ptr
from . import delays as _delays


# 16-bit sweep input: int16 storage (values 0..1023 have the same bits) or
# torch.uint16 where this torch has it
_U16_TYPES = tuple(t for t in (torch.int16, getattr(torch, "uint16", None)) if t is not None)
_CODE_OF = {"f32": _lib.F32, "u8": _lib.U8, "u16": _lib.U16}


def _is_int_pad(padval):
    if isinstance(padval, str):
        return padval == "rotate"
    return float(padval).is_integer() and 0 <= float(padval) <= 255


def _pads16(x, C, padval):
    """(pad mode, per-channel pad values) of a 16-bit sweep."""
    if isinstance(padval, str):
        if padval != "rotate":
            raise ValueError("16-bit sweep input takes integer or 'rotate' pads")
        return _lib.PAD_ROTATE, None
    if not (float(padval).is_integer() and 0 <= float(padval) <= 1023):
        raise ValueError("16-bit sweep pads must be integers in [0, 1023]")
    return _lib.PAD_VALUE, torch.full((C,), float(padval), dtype=torch.float32, device=x.device)


def _is_int_pad16(padval):
    """Pads the 16-bit sweep can bake in exactly (integers <= 1023, 'rotate')."""
    if isinstance(padval, str):
        return padval == "rotate"
    return float(padval).is_integer() and 0 <= float(padval) <= 1023


# Test switches applied to every sweep plan this process creates (parity
# tests set them, e.g. with pytest's monkeypatch.setitem; production code
# never does): poison -- factorised plans fill their pattern image with 0xFF
# bytes before stage 1 (pdd_sweep_plan_set_poison); segment_bytes > 0 -- the
# scratch budget of one time segment (pdd_sweep_plan_set_segment_bytes);
# no_skew -- factorised plans are created with plane-aligned tiles
# (PDD_SWEEP_NO_SKEW; bench.py --no-skew, the A/B of DESIGN.md §3.2).
TEST_SWITCHES = {"poison": False, "segment_bytes": 0, "no_skew": False}


def _apply_test_switches(p):
    if TEST_SWITCHES["poison"]:
        _lib.check(_lib.lib().pdd_sweep_plan_set_poison(p, 1), "pdd_sweep_plan_set_poison")
    if TEST_SWITCHES["segment_bytes"]:
        _lib.check(_lib.lib().pdd_sweep_plan_set_segment_bytes(p, int(TEST_SWITCHES["segment_bytes"])),
                   "pdd_sweep_plan_set_segment_bytes")


class DMSweep(object):
    """A reusable sweep plan: ``DMSweep(dms, freqs, dt)(x)`` -> device plane.

    dtype: 'f32' (float32 input), 'u8' (8-bit filterbank input; exact
    integer accumulation) or 'u16' (16-bit samples <= 1023, e.g. the offset
    integer zero-DM + downsample prologue of the stream; exact).  ``x`` is a
    [C, N] device tensor of that dtype (int16 / uint16 storage for 'u16') or
    a ``Spectra``."""

    def __init__(self, dms, freqs, dt, cur_dm=0.0, dtype="f32", input_max=None, factor=True,
                 skew=True):
        """``input_max`` (integer dtypes): the largest sample value the input
        and its integer pads hold (default 255 for 'u8', 1023 for 'u16'); a
        tighter bound lets the exact packed-u16 accumulation convert less
        often (pdd_sweep_plan_set_input_max).  ``factor``: 8-bit plans may
        sweep exactly factorised over groups of 4 channels when that pays
        (pdd_sweep_plan_create_ex PDD_SWEEP_FACTOR; bit-identical planes);
        False forces the channel-by-channel kernel; 2 or 4: that group size
        only (still where it pays); "force2" / "force4" (= "force"): that
        group size wherever the windows fit, paying or not (tests).
        ``skew``: factorised plans use delay-aligned time tiles (each trial's
        tile skewed by its delay at a mid-band group: fewer staged window
        elements, the same plane); False keeps plane-aligned tiles
        (PDD_SWEEP_NO_SKEW; A/B measurements and parity tests)."""
        _lib.require_gpu()
        self.dms = np.atleast_1d(np.asarray(dms, dtype=np.float64))
        self.freqs = np.asarray(freqs, dtype=np.float64)
        self.dt = dt
        self.cur_dm = cur_dm
        assert np.all(self.dms >= 0)
        table = _delays.sweep_table(self.dms, self.freqs, dt, cur_dm)
        self.table = _delays.to_int32(table)
        self.D, self.C = self.table.shape
        self.max_bin = int(self.table.max()) if self.table.size else 0
        self.dtype = dtype
        self.input_max = None if input_max is None else int(input_max)
        if factor == "force":
            factor = "force4"
        assert factor in (True, False, 2, 4, "force2", "force4"), "bad factor %r" % (factor,)
        self.factor = factor
        self.skew = bool(skew)
        if self.input_max is not None:
            assert dtype in ("u8", "u16") and 1 <= self.input_max <= (255 if dtype == "u8" else 1023)
        self._plans = {}

    def _plan(self, code):
        p = self._plans.get(code)
        if p is None:
            h = ctypes.c_void_p()
            tab = np.ascontiguousarray(self.table)
            _lib.check(_lib.lib().pdd_sweep_plan_create_ex(
                tab.ctypes.data_as(ctypes.c_void_p), self.D, self.C, code,
                self._factor_flags(), ctypes.byref(h)),
                "pdd_sweep_plan_create_ex")
            p = h
            self._plans[code] = p
            _apply_test_switches(p)
            if self.input_max is not None and code != _lib.F32:
                _lib.check(_lib.lib().pdd_sweep_plan_set_input_max(p, self.input_max),
                           "pdd_sweep_plan_set_input_max")
        return p

    def set_segment_bytes(self, nbytes, code=None):
        """Scratch budget of one time segment of this sweep's plans (0 = the
        library default); tests of the multi-segment path on small blocks."""
        codes = [code] if code is not None else list(self._plans)
        for c in codes:
            _lib.check(_lib.lib().pdd_sweep_plan_set_segment_bytes(self._plan(c), int(nbytes)),
                       "pdd_sweep_plan_set_segment_bytes")

    def info(self, code=_lib.F32):
        a = np.zeros(8, dtype=np.int64)
        _lib.check(_lib.lib().pdd_sweep_plan_info(self._plan(code), a.ctypes.data_as(ctypes.c_void_p)),
                   "pdd_sweep_plan_info")
        keys = ("D", "C", "dms_per_block", "samples_per_block", "lds_bytes", "max_bin", "min_bin",
                "variant")
        return dict(zip(keys, (int(v) for v in a)))

    def _factor_flags(self):
        f = self.factor
        if f is False:
            return 0
        flags = _lib.SWEEP_FACTOR
        if not getattr(self, "skew", True) or TEST_SWITCHES["no_skew"]:
            flags |= _lib.SWEEP_NO_SKEW
        if isinstance(f, str):
            flags |= _lib.SWEEP_FACTOR_FORCE
            f = int(f[-1])
        if f is not True:
            flags |= _lib.SWEEP_FACTOR_G2 if f == 2 else _lib.SWEEP_FACTOR_G4
        return flags

    def factor_info(self, code=_lib.U8):
        """(channels per factor group, stage-1 patterns) of the plan for
        ``code``; (0, 0) for a channel-by-channel plan."""
        n = ctypes.c_int64(0)
        g = _lib.lib().pdd_sweep_plan_factor(self._plan(code), ctypes.byref(n))
        if g < 0:
            _lib.check(g, "pdd_sweep_plan_factor")
        return int(g), int(n.value)

    def skew_info(self, code=_lib.U8):
        """(largest per-trial tile skew, extra time tiles per segment) of the
        plan for ``code``: (0, 0) for plane-aligned tiles (pdd_sweep_plan_skew)."""
        n = ctypes.c_int64(0)
        s = _lib.lib().pdd_sweep_plan_skew(self._plan(code), ctypes.byref(n))
        if s < 0:
            _lib.check(s, "pdd_sweep_plan_skew")
        return int(s), int(n.value)

    def n_out(self, N, trim=True):
        if trim and self.max_bin > 0:
            return max(0, N - self.max_bin)
        return N

    def __call__(self, x, padval=0, trim=True, out=None, stream=None, n_out=None, out_bias=0.0):
        """Sweep ``x`` into ``out`` (allocated if None).  ``n_out`` (optional)
        is the number of plane columns to produce; the default is this grid's
        trimmed width ``n_out(N, trim)``.  A caller sweeping a slice of a
        larger grid passes the GLOBAL width (<= this slice's), so every rank
        of a DM-sharded sweep fills identically shaped rows; columns past a
        row's own trimmed length are the reference's padded values
        (dedisperse(trim=False) semantics), never out-of-bounds reads.
        ``out_bias`` is added to every plane value (an offset encoding of the
        input, e.g. -offset * C for the u16 prologue; exact for integers)."""
        from .formats.spectra import Spectra, _pad_args
        f32 = None
        if isinstance(x, Spectra):
            assert x.numchans == self.C
            f32 = x.device_data
            raw8 = x._raw8
            x = raw8 if (self.dtype == "u8" and raw8 is not None) else f32
        if x.dim() != 2 or x.shape[0] != self.C:
            raise ValueError("expected a [C=%d, N] device tensor" % self.C)
        if x.stride(1) != 1:
            x = x.contiguous()
        N = x.shape[1]
        if n_out is None:
            n_out = self.n_out(N, trim)
        else:
            n_out = int(n_out)
            if not 0 <= n_out <= N:
                raise ValueError("n_out=%d outside [0, N=%d]" % (n_out, N))
        if out is None:
            out = torch.empty((self.D, n_out), dtype=torch.float32, device=x.device)
        if out.shape[0] != self.D or out.shape[1] < n_out or out.stride(1) != 1:
            raise ValueError("out must be [D=%d, >= %d] with unit column stride, got %s / %s"
                             % (self.D, n_out, tuple(out.shape), tuple(out.stride())))
        if n_out == 0 or N == 0:
            return out
        if x.dtype == torch.uint8 and not _is_int_pad(padval):
            # fractional / statistical pads need the float32 image
            if f32 is None:
                f32 = torch.empty((self.C, N), dtype=torch.float32, device=x.device)
                call("pdd_convert_f32", ptr(x), _lib.U8, self.C, N, x.stride(0), ptr(f32), N,
                     stream_ptr(stream))
            x = f32
        if x.dtype == torch.uint8:
            code = _lib.U8
            if isinstance(padval, str):
                mode, pv = _lib.PAD_ROTATE, None
            else:
                mode = _lib.PAD_VALUE
                pv = torch.full((self.C,), float(padval), dtype=torch.float32, device=x.device)
        elif x.dtype in _U16_TYPES:
            code = _lib.U16
            mode, pv = _pads16(x, self.C, padval)
        elif x.dtype == torch.float32:
            code = _lib.F32
            mode, pv = _pad_args(x, padval)
        else:
            raise TypeError("sweep input must be float32, uint8 or 16-bit")
        if code != _lib.F32 and self.input_max is not None and mode == _lib.PAD_VALUE \
                and float(padval) > self.input_max:
            # the packed-u16 flush interval assumes every summed value <= input_max
            raise ValueError("pad %g above the sweep's input bound %d" % (float(padval),
                                                                         self.input_max))
        call("pdd_sweep_execute_ex", self._plan(code), ptr(x), N, x.stride(0), 0, 0, mode, ptr(pv),
             ptr(out), out.stride(0), n_out, float(out_bias), stream_ptr(stream))
        return out

    def sweep_ds(self, x8, ds, padval=0, out=None, n_out=None, stream=None):
        """Sweep ``Spectra.downsample(ds)`` of the 8-bit rows ``x8`` ([C,
        n_raw] uint8) without forming the downsampled copy: the co-adds (<=
        1020, exact) are formed by the interleave pre-pass of the 16-bit sweep
        (pdd_sweep_execute_ds; dtype='u16' plans, ds 2..4).  Pads act on the
        downsampled series (integers <= 1023 or 'rotate')."""
        if self.dtype != "u16":
            raise TypeError("sweep_ds needs a dtype='u16' DMSweep")
        mode, pv = _pads16(x8, self.C, padval)
        N = x8.shape[1] // int(ds)
        n_out = self.n_out(N, True) if n_out is None else int(n_out)
        if out is None:
            out = torch.empty((self.D, max(n_out, 1)), dtype=torch.float32, device=x8.device)
        assert x8.dtype == torch.uint8 and x8.dim() == 2 and x8.shape[0] == self.C
        assert x8.stride(1) == 1 and out.shape[0] == self.D and out.shape[1] >= n_out
        assert out.stride(1) == 1
        call("pdd_sweep_execute_ds", self._plan(_lib.U16), ptr(x8), x8.shape[1], x8.stride(0),
             int(ds), mode, ptr(pv), ptr(out), out.stride(0), n_out, 0, 1, stream_ptr(stream))
        return out

    def sweep_pieces(self, xp, N, piece, x_off, n_out, out, stream=None):
        """Plane columns [x_off, x_off + n_out) of the sweep of a block held
        in the "pieces" layout an all-gather of channel-major time slices
        produces: ``xp`` memory = [ceil(N/piece)][C][piece] (piece a power of
        two), sample s of channel c at xp[(s//piece)*C*piece + c*piece +
        s%piece] (pdd_sweep_execute_ex).  Pads are value 0 (trim=True grids
        with delays >= 0 never read them)."""
        code = _lib.U8 if xp.dtype == torch.uint8 else _lib.F32
        if code == _lib.U8 and self.dtype != "u8":
            raise TypeError("8-bit pieces need a dtype='u8' DMSweep")
        assert out.shape[0] == self.D and out.shape[1] >= n_out and out.stride(1) == 1
        assert xp.is_contiguous() and xp.numel() >= -(-N // piece) * self.C * piece
        pv = torch.zeros(self.C, dtype=torch.float32, device=xp.device)
        call("pdd_sweep_execute_ex", self._plan(code), ptr(xp), N, 0, piece, x_off, _lib.PAD_VALUE,
             ptr(pv), ptr(out), out.stride(0), n_out, 0.0, stream_ptr(stream))
        return out

    def pattern_bytes(self, n_out, code=_lib.U8):
        """Bytes of the pattern image one staged launch of ``n_out`` columns
        needs (0: not a factorised plan; pdd_sweep_pattern_bytes)."""
        return int(_lib.lib().pdd_sweep_pattern_bytes(self._plan(code), int(n_out)))

    def sweep_pieces_stage(self, xp, N, piece, x_off, n_out, out, patterns, stage, stream=None):
        """Stage 1 (the pattern image into ``patterns``, a uint8 device
        buffer of >= pattern_bytes(n_out)), stage 2 (the sweep of that image
        into ``out``) or both (3) of sweep_pieces on a factorised plan
        (pdd_sweep_execute_stage): stage 1 of the next block can run on one
        stream while stage 2 of this one runs on another."""
        code = _lib.U8 if xp.dtype == torch.uint8 else _lib.F32
        assert out is None or (out.shape[0] == self.D and out.shape[1] >= n_out
                               and out.stride(1) == 1)
        assert patterns.is_cuda and patterns.is_contiguous()
        nbytes = patterns.numel() * patterns.element_size()
        # (the zero pads are allocated once: a fill kernel on torch's default
        # stream would serialise the CU-partitioned streams of a pipeline)
        pv = getattr(self, "_pv0", None)
        if pv is None or pv.device != xp.device:
            pv = self._pv0 = torch.zeros(self.C, dtype=torch.float32, device=xp.device)
        ld = 0 if piece else xp.stride(0)  # piece 0: channel-major [C][ld] rows
        call("pdd_sweep_execute_stage", self._plan(code), ptr(xp), N, ld, piece, x_off,
             _lib.PAD_VALUE, ptr(pv), ptr(out), out.stride(0) if out is not None else 0, n_out,
             0.0, ptr(patterns), nbytes, int(stage), stream_ptr(stream))
        return out

    def set_timing(self, on=True, code=None):
        """Bracket the sweep kernel of every execute with HIP events (on the
        execute stream); read the last duration with kernel_ms()."""
        code = _CODE_OF[self.dtype] if code is None else code
        _lib.check(_lib.lib().pdd_sweep_set_timing(self._plan(code), int(bool(on))),
                   "pdd_sweep_set_timing")
        self._timed_code = code

    def kernel_ms(self):
        """Sum of the bracketed sweep-kernel durations since the last read."""
        return self.timing_read()[0]

    def timing_read(self):
        """(sum of the bracketed sweep-kernel durations in ms, launches) since
        the last read; every launch has its own HIP event pair on the stream
        it ran on, recorded without host synchronisation."""
        v = ctypes.c_float()
        n = ctypes.c_int64()
        _lib.check(_lib.lib().pdd_sweep_timing_read(self._plan(self._timed_code), ctypes.byref(v),
                                                    ctypes.byref(n)), "pdd_sweep_timing_read")
        return float(v.value), int(n.value)

    def close(self):
        for p in self._plans.values():
            _lib.lib().pdd_sweep_plan_destroy(p)
        self._plans = {}

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def execute_plan(spectra, ddplan, padval=0, trim=True):
    """Run a DDplan (pypulsar_amd.utils.ddplan.DDplan) over a Spectra.

    Per DDstep: downsample by step.downsamp (Spectra.downsample semantics),
    then -- without subbands -- one DM sweep over step.DMs, or -- with
    subbands -- for each subband pass k: Spectra.subband(nsub, subDM_k,
    padval) with subDM_k = loDM + (k+0.5)*dsubDM, then a DM sweep of that
    pass's DMs over the subbands.  Returns [(step, [(dms, plane), ...])].
    Order decision: downsample BEFORE subbanding (4x less stage-1 work at
    downsamp 4)."""
    import copy
    results = []
    for step in ddplan.DDsteps:
        base = copy.deepcopy(spectra)
        if step.downsamp > 1:
            base.downsample(step.downsamp)
        outs = []
        for subdm, dms in step.subband_calls():
            if subdm is None:
                s = base
            else:
                s = copy.deepcopy(base)
                s.subband(step.numsub, subdm, padval=padval)
            sw = DMSweep(dms, s.freqs, s.dt, cur_dm=s.dm,
                         dtype="u8" if s._raw8 is not None else "f32")
            outs.append((dms, sw(s, padval=padval, trim=trim)))
            sw.close()
        results.append((step, outs))
    return results


class GroupedSweep(object):
    """One launch for ``n_grp`` independent sweeps over contiguous channel
    groups: group g sweeps channels g*C .. g*C + C - 1 of the input with its
    own [D][C] delay table; trial d of group g lands in plane row
    g*row_g + d*row_d (pdd_sweep_plan_create_grouped / _execute_grouped)."""

    def __init__(self, tables, dtype="f32"):
        _lib.require_gpu()
        t = np.ascontiguousarray(_delays.to_int32(np.asarray(tables)))
        assert t.ndim == 3, "tables must be [n_grp, D, C]"
        self.n_grp, self.D, self.C = t.shape
        self.max_bin = int(t.max()) if t.size else 0
        self.dtype = dtype
        code = _CODE_OF[dtype]
        h = ctypes.c_void_p()
        _lib.check(_lib.lib().pdd_sweep_plan_create_grouped(
            t.ctypes.data_as(ctypes.c_void_p), self.n_grp, self.D, self.C, code, ctypes.byref(h)),
            "pdd_sweep_plan_create_grouped")
        self._plan = h

    def __call__(self, x, n_out, out, row_g, row_d, pad_mode=_lib.PAD_VALUE, padvals=None,
                 stream=None):
        assert x.dim() == 2 and x.shape[0] == self.n_grp * self.C and x.stride(1) == 1
        if pad_mode == _lib.PAD_VALUE and padvals is None:
            padvals = torch.zeros(x.shape[0], dtype=torch.float32, device=x.device)
        call("pdd_sweep_execute_grouped", self._plan, ptr(x), x.shape[1], x.stride(0), pad_mode,
             ptr(padvals), ptr(out), out.stride(0), n_out, row_g, row_d, stream_ptr(stream))
        return out

    def info(self):
        """Plan extents (pdd_sweep_plan_info) as a dict (DMs per block, ...)."""
        a = np.zeros(8, dtype=np.int64)
        _lib.check(_lib.lib().pdd_sweep_plan_info(self._plan, a.ctypes.data_as(ctypes.c_void_p)),
                   "pdd_sweep_plan_info")
        keys = ("D", "C", "dms_per_block", "samples_per_block", "lds_bytes", "max_bin", "min_bin",
                "variant")
        return dict(zip(keys, (int(v) for v in a)))

    def set_timing(self, on=True):
        """Bracket every sweep-kernel launch of this plan with a HIP event pair."""
        _lib.check(_lib.lib().pdd_sweep_set_timing(self._plan, int(bool(on))),
                   "pdd_sweep_set_timing")

    def timing_read(self):
        """(summed kernel ms, launches) since set_timing / the last read."""
        v = ctypes.c_float(0.0)
        n = ctypes.c_int64(0)
        _lib.check(_lib.lib().pdd_sweep_timing_read(self._plan, ctypes.byref(v), ctypes.byref(n)),
                   "pdd_sweep_timing_read")
        return float(v.value), int(n.value)

    def execute_ds(self, x8, ds, n_out, out, row_g, row_d, pad_mode=_lib.PAD_VALUE, padvals=None,
                   stream=None):
        """The grouped sweep of ``x8`` ([n_grp*C, n_raw] uint8) downsampled by
        ``ds`` (2..4) on the fly (pdd_sweep_execute_ds; dtype='u16' plans)."""
        assert self.dtype == "u16", "execute_ds needs a dtype='u16' GroupedSweep"
        assert x8.dtype == torch.uint8 and x8.dim() == 2 and x8.shape[0] == self.n_grp * self.C
        assert x8.stride(1) == 1
        if pad_mode == _lib.PAD_VALUE and padvals is None:
            padvals = torch.zeros(x8.shape[0], dtype=torch.float32, device=x8.device)
        call("pdd_sweep_execute_ds", self._plan, ptr(x8), x8.shape[1], x8.stride(0), int(ds),
             pad_mode, ptr(padvals), ptr(out), out.stride(0), n_out, row_g, row_d,
             stream_ptr(stream))
        return out

    def close(self):
        if self._plan is not None:
            _lib.lib().pdd_sweep_plan_destroy(self._plan)
            self._plan = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _Step(object):
    """Device plans + buffers of one DDstep (DDplanExecutor)."""
    pass


class DDplanExecutor(object):
    """Two-stage DDplan executor whose delay tables, sweep plans and device
    buffers are built ONCE per (plan, channel frequencies, dt, N) -- the
    reference computes its delays on the host per call
    (formats/spectra.py:126-130, 247-250); here every call of the executor only
    launches kernels (no host table work, no synchronous hipMemcpy).

    Per DDstep (DDplan2b.py:102-199), ``trim=True``:
      * downsample by ``step.downsamp`` (Spectra.downsample, spectra.py:329-351;
        the raw 8-bit rows when the Spectra still holds them: exact integer
        sums from a quarter of the bytes);
      * without subbands: one DMSweep over ``step.DMs``;
      * with subbands: stage 1 forms every pass's subbands in ONE grouped
        launch -- one group per subband (its C/nsub channels) whose trials are
        the passes' subDMs (Spectra.subband shifts + group sum,
        spectra.py:96-138; pads as there, full length) -- and stage 2 sweeps
        every pass's DMs in ONE grouped launch -- one group per pass, whose
        channels are that pass's subbands at their centre frequencies
        (Spectra.dedisperse(dm, padval, trim=True) + channel sum, with the
        pads of the subbanded data).  subDM_k = loDM + (k+0.5)*dsubDM.

    ``__call__(spectra, padval)`` returns [(step, dms, plane)], plane rows =
    the step's DMs, columns = the common prefix of the per-DM trimmed series.
    The planes are the executor's own buffers, overwritten by the next call.
    """

    def __init__(self, ddplan, freqs, dt, N, cur_dm=0.0, raw8=False, device="cuda"):
        _lib.require_gpu()
        self.freqs = np.asarray(freqs, dtype=np.float64)
        self.C = len(self.freqs)
        self.N = int(N)
        self.dt = dt
        self.cur_dm = cur_dm
        self.device = torch.device(device)
        self.steps = []
        for step in ddplan.DDsteps:
            s = _Step()
            s.step = step
            s.ds = int(step.downsamp)
            s.dt = dt * s.ds
            s.n_ds = self.N // s.ds if s.ds > 1 else self.N
            # 8-bit rows downsampled by <= 4 stay exact integers <= 1020: the
            # co-add is kept as uint16 and swept on the 16-bit path
            s.u16 = bool(raw8) and 1 < s.ds <= 4
            s.x = None      # float32 image of a downsampled step (allocated on use)
            calls = step.subband_calls()
            s.two_stage = calls[0][0] is not None
            if not s.two_stage:
                # 8-bit rows at full rate go through the exact u16 sweep
                s.sw = DMSweep(step.DMs, self.freqs, s.dt, cur_dm=cur_dm,
                               dtype="u8" if (raw8 and s.ds == 1) else ("u16" if s.u16 else "f32"))
                s.n_out = s.sw.n_out(s.n_ds, True)
                s.plane = torch.empty((s.sw.D, max(s.n_out, 1)), dtype=torch.float32,
                                      device=self.device)
                self.steps.append(s)
                continue
            nsub = step.numsub
            cps = self.C // nsub
            subdms = [c[0] for c in calls]
            ncall = len(calls)
            # stage 1: [nsub groups][ncall trials][cps channels]
            t1 = np.stack([_delays.subband_bins(sd, self.freqs, s.dt, nsub, cur_dm=cur_dm)
                           for sd in subdms])                      # [ncall, C]
            s.t1 = t1.reshape(ncall, nsub, cps).transpose(1, 0, 2)  # [nsub, ncall, cps]
            # 8-bit rows: stage 1 on the exact integer path (u8 at the raw
            # rate, u16 co-adds at ds <= 4)
            s.int1 = "u8" if (raw8 and s.ds == 1) else ("u16" if s.u16 else None)
            s.g1 = GroupedSweep(s.t1, s.int1 or "f32")
            s.sub = None    # subband plane (only when the stages are not chained)
            s.chain, s.chain_pads = True, None
            # stage 2: [ncall groups][per-call DMs][nsub subbands at their centres]
            _, _, ctr = _delays.subband_layout(self.freqs, nsub)
            per = len(calls[0][1])
            assert all(len(c[1]) == per for c in calls)
            t2 = np.stack([_delays.sweep_table(c[1], ctr, s.dt, cur_dm=cur_dm) for c in calls])
            s.g2 = GroupedSweep(t2, "f32")
            s.nsub, s.ncall, s.per = nsub, ncall, per
            s.n_out = max(0, s.n_ds - max(0, s.g2.max_bin))
            s.plane = torch.empty((ncall * per, max(s.n_out, 1)), dtype=torch.float32,
                                  device=self.device)
            self.steps.append(s)

    def __call__(self, spectra, padval=0):
        from .formats.spectra import _pad_args
        src = spectra.device_data
        assert tuple(src.shape) == (self.C, self.N), "executor built for a [%d, %d] Spectra" % (
            self.C, self.N)
        assert spectra.dm == self.cur_dm and spectra.dt == self.dt
        raw8 = getattr(spectra, "_raw8", None)
        if raw8 is not None and (tuple(raw8.shape) != tuple(src.shape) or raw8.stride(1) != 1):
            raw8 = None
        results = []
        for s in self.steps:
            # the exact 16-bit path needs the raw 8-bit rows and integer pads
            use16 = s.u16 and raw8 is not None and _is_int_pad16(padval)
            use8 = (s.two_stage and s.int1 == "u8" and raw8 is not None
                    and _is_int_pad(padval))
            if s.ds > 1 and use16:
                # the 16-bit sweeps co-add the raw rows in their interleave
                # pre-pass (pdd_sweep_execute_ds): no downsampled copy
                x = raw8
            elif s.ds > 1:
                if s.x is None:
                    s.x = torch.empty((self.C, s.n_ds), dtype=torch.float32, device=self.device)
                x = s.x
                if s.n_ds and raw8 is not None:
                    call("pdd_downsample_u8", ptr(raw8), self.C, self.N, raw8.stride(0), s.ds,
                         ptr(x), s.n_ds, stream_ptr())
                elif s.n_ds:
                    call("pdd_downsample", ptr(src), self.C, self.N, src.stride(0), s.ds, ptr(x),
                         s.n_ds, stream_ptr())
            else:
                x = raw8 if use8 else src
            if not s.two_stage:
                sw = s.sw
                if sw.dtype == "u8" and raw8 is not None and _is_int_pad(padval):
                    x = raw8
                elif sw.dtype == "u16" and use16:
                    sw.sweep_ds(x, s.ds, padval=padval, out=s.plane, n_out=s.n_out)
                    results.append((s.step, s.step.DMs, s.plane[:, :s.n_out]))
                    continue
                elif sw.dtype != "f32":
                    # pads that are not small integers (or no raw rows): float image
                    if getattr(s, "sw_f32", None) is None:
                        s.sw_f32 = DMSweep(s.step.DMs, self.freqs, s.dt, cur_dm=self.cur_dm,
                                           dtype="f32")
                    sw = s.sw_f32
                sw(x, padval=padval, trim=True, out=s.plane)
                results.append((s.step, s.step.DMs, s.plane[:, :s.n_out]))
                continue
            g1 = s.g1
            if s.int1 and not (use16 or use8):
                if getattr(s, "g1_f32", None) is None:
                    s.g1_f32 = GroupedSweep(s.t1, "f32")
                g1 = s.g1_f32
            if (use16 or use8) and not isinstance(padval, str) and s.chain:
                # both stages chained: stage 1 writes stage 2's input image
                # directly (pdd_subband_chain), no subband plane
                if s.n_out:
                    if s.chain_pads is None or s.chain_pads[0] != float(padval):
                        s.chain_pads = (float(padval),
                                        torch.full((self.C,), float(padval), dtype=torch.float32,
                                                   device=self.device),
                                        torch.full((s.ncall * s.nsub,), float(padval),
                                                   dtype=torch.float32, device=self.device))
                    _, pv1, pv2 = s.chain_pads
                    rc = _lib.lib().pdd_subband_chain(
                        g1._plan, ptr(raw8), self.N, raw8.stride(0), s.ds, _lib.PAD_VALUE,
                        ptr(pv1), s.g2._plan, ptr(pv2), ptr(s.plane), s.plane.stride(0),
                        s.n_out, s.per, 1, stream_ptr())
                    if rc != _lib.ENOCHAIN:
                        _lib.check(rc, "pdd_subband_chain")   # errors (e.g. -2 OOM) raise
                        results.append((s.step, s.step.DMs, s.plane[:, :s.n_out]))
                        continue
                    # a geometry the chain does not take (nothing was
                    # launched): run the stages apart from now on
                    s.chain = False
            if s.sub is None:
                s.sub = torch.empty((s.ncall * s.nsub, s.n_ds), dtype=torch.float32,
                                    device=self.device)
            if use16 or use8:
                pv = torch.full((x.shape[0],), float(padval), dtype=torch.float32,
                                device=x.device) if not isinstance(padval, str) else None
                mode = _lib.PAD_ROTATE if isinstance(padval, str) else _lib.PAD_VALUE
            else:
                mode, pv = _pad_args(x, padval)
            if use16 and s.ds > 1:
                g1.execute_ds(x, s.ds, s.n_ds, s.sub, row_g=1, row_d=s.nsub, pad_mode=mode,
                              padvals=pv)
            else:
                g1(x, s.n_ds, s.sub, row_g=1, row_d=s.nsub, pad_mode=mode, padvals=pv)
            if s.n_out:
                # stage 2 pads: those of each pass's subbanded Spectra
                # (dedisperse(dm, padval) on the subbanded data)
                mode2, pv2 = _pad_args(s.sub, padval)
                s.g2(s.sub, s.n_out, s.plane, row_g=s.per, row_d=1, pad_mode=mode2, padvals=pv2)
            results.append((s.step, s.step.DMs, s.plane[:, :s.n_out]))
        return results

    def close(self):
        for s in self.steps:
            for name in ("sw", "sw_f32", "g1", "g1_f32", "g2"):
                obj = getattr(s, name, None)
                if obj is not None:
                    obj.close()


def execute_plan_grouped(spectra, ddplan, padval=0):
    """One-off two-stage DDplan execution (DDplanExecutor built for this
    Spectra, run once; the returned planes are its own buffers).  Callers
    that execute the same plan repeatedly keep a DDplanExecutor instead."""
    ex = DDplanExecutor(ddplan, spectra.freqs, spectra.dt, spectra.numspectra,
                        cur_dm=spectra.dm, raw8=getattr(spectra, "_raw8", None) is not None)
    out = ex(spectra, padval=padval)
    ex.close()
    return out


def cu_masked_stream(cus, device=None):
    """A torch ExternalStream whose kernels run only on the compute units in
    ``cus`` (pdd_stream_create_cu_mask / hipExtStreamCreateWithCUMask); the
    HIP stream lives until cu_stream_release(stream)."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    n = max(cus) // 32 + 1
    words = np.zeros(max(n, 8), dtype=np.uint32)
    for c in cus:
        words[c // 32] |= np.uint32(1 << (c % 32))
    h = ctypes.c_void_p()
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().pdd_stream_create_cu_mask(words.ctypes.data_as(ctypes.c_void_p),
                                                        len(words), ctypes.byref(h)),
                   "pdd_stream_create_cu_mask")
        st = torch.cuda.ExternalStream(h.value, device=dev)
    st._pdd_handle = h
    return st


def cu_stream_release(st):
    h = getattr(st, "_pdd_handle", None)
    if h is not None and h.value:
        _lib.check(_lib.lib().pdd_stream_destroy(h), "pdd_stream_destroy")
        st._pdd_handle = None
