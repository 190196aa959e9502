"""ctypes binding of libpdd.so (the C ABI declared in include/pdd.h).

The HIP library is REQUIRED: there is no CPU fallback anywhere in the product
path.  If ``libpdd.so`` is missing, ``lib()`` raises ``PddLibraryMissing``.
torch is imported first so that libpdd.so binds to the HIP runtime torch has
already loaded (both carry the SONAME ``libamdhip64.so.7``): device pointers
and stream handles are shared with torch.
"""
import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime before libpdd.so)

from . import _digest

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libpdd.so")
# developer builds (-DPDD_SWEEP_DEV, scripts/build_dev.sh) are loaded from
# PDD_DEV_LIB for timing experiments (no digest check); production runs
# never set it
_DEV_LIB = os.environ.get("PDD_DEV_LIB")
if _DEV_LIB:
    LIB_PATH = _DEV_LIB

# element types / modes (include/pdd.h)
F32, U8, U16 = 0, 1, 2
PAD_VALUE, PAD_ROTATE = 0, 1
STAT_MEAN, STAT_MEDIAN, STAT_STD, STAT_MIN, STAT_MAX = 0, 1, 2, 3, 4
LAYOUT_TIME_MAJOR, LAYOUT_CHAN_MAJOR = 0, 1
ENOCHAIN = -5          # pdd_subband_chain: geometry does not chain (nothing launched)
ZDM_NONE, ZDM_INT, ZDM_WRAP = 0, 1, 2
SWEEP_FACTOR = 1       # pdd_sweep_plan_create_ex: exact factorised 8-bit sweeps allowed
SWEEP_FACTOR_FORCE = 2  # ... and taken whenever the windows fit (tests)
SWEEP_FACTOR_G2 = 4     # ... over groups of 2 channels only
SWEEP_FACTOR_G4 = 8     # ... over groups of 4 channels only
SWEEP_NO_SKEW = 16      # ... with plane-aligned (not delay-aligned) factorised tiles

# every symbol include/pdd.h declares (checked by tests/test_abi.py)
EXPORTS = (
    "pdd_version", "pdd_last_error", "pdd_sync", "pdd_corner_turn", "pdd_convert_f32",
    "pdd_channel_stats", "pdd_shift_pad", "pdd_shift_group_sum", "pdd_downsample",
    "pdd_zero_dm", "pdd_sweep_plan_create", "pdd_sweep_execute", "pdd_sweep_plan_info",
    "pdd_sweep_plan_set_input_max",
    "pdd_sweep_plan_destroy", "pdd_global_stats", "pdd_scale_rows", "pdd_masked_fill",
    "pdd_smooth", "pdd_zdm_downsample", "pdd_sweep_set_timing", "pdd_sweep_kernel_ms",
    "pdd_sweep_plan_create_grouped", "pdd_sweep_execute_grouped", "pdd_sp_chunk_stats",
    "pdd_sp_search", "pdd_psrfits_subints", "pdd_downsample_u8", "pdd_sweep_timing_read",
    "pdd_sweep_execute_ex", "pdd_zdm_int_downsample", "pdd_downsample_u8_u16",
    "pdd_sweep_execute_ds", "pdd_subband_chain", "pdd_scratch_release",
    "pdd_sweep_plan_create_ex", "pdd_sweep_plan_factor", "pdd_sweep_plan_skew", "pdd_source_digest",
    "pdd_sweep_plan_set_poison", "pdd_sweep_plan_set_segment_bytes",
    "pdd_sweep_pattern_bytes", "pdd_sweep_execute_stage", "pdd_stream_create_cu_mask",
    "pdd_stream_destroy",
)


def source_digest():
    """Digest of the library sources + build flags in this tree
    (pypulsar_amd/_digest.py); a loaded library must carry the same."""
    return _digest.source_digest()


class PddLibraryMissing(RuntimeError):
    pass


class PddError(RuntimeError):
    pass


_lib = None

_vp, _i64, _int = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
_SIGS = {
    "pdd_version": ([], _int),
    "pdd_source_digest": ([], ctypes.c_char_p),
    "pdd_sweep_plan_set_poison": ([_vp, _int], _int),
    "pdd_sweep_plan_set_segment_bytes": ([_vp, _i64], _int),
    "pdd_last_error": ([], ctypes.c_char_p),
    "pdd_sync": ([_vp], _int),
    "pdd_scratch_release": ([], _int),
    "pdd_corner_turn": ([_vp, _int, _i64, _i64, _i64, _vp, _int, _i64, _vp], _int),
    "pdd_convert_f32": ([_vp, _int, _i64, _i64, _i64, _vp, _i64, _vp], _int),
    "pdd_channel_stats": ([_vp, _i64, _i64, _i64, _int, _vp, _vp], _int),
    "pdd_shift_pad": ([_vp, _i64, _i64, _i64, _vp, _int, _vp, _vp, _i64, _i64, _vp], _int),
    "pdd_shift_group_sum": ([_vp, _i64, _i64, _i64, _vp, _int, _vp, _i64, _vp, _i64, _i64, _vp],
                            _int),
    "pdd_downsample": ([_vp, _i64, _i64, _i64, _i64, _vp, _i64, _vp], _int),
    "pdd_downsample_u8": ([_vp, _i64, _i64, _i64, _i64, _vp, _i64, _vp], _int),
    "pdd_downsample_u8_u16": ([_vp, _i64, _i64, _i64, _i64, _vp, _i64, _vp], _int),
    "pdd_zero_dm": ([_vp, _int, _i64, _i64, _i64, _int, _vp, _i64, _vp], _int),
    "pdd_sweep_plan_create": ([_vp, _i64, _i64, _int, ctypes.POINTER(_vp)], _int),
    "pdd_sweep_plan_create_ex": ([_vp, _i64, _i64, _int, _int, ctypes.POINTER(_vp)], _int),
    "pdd_sweep_plan_factor": ([_vp, _vp], _int),
    "pdd_sweep_plan_skew": ([_vp, _vp], _int),
    "pdd_sweep_execute": ([_vp, _vp, _i64, _i64, _int, _vp, _vp, _i64, _i64, _vp], _int),
    "pdd_sweep_execute_ex": ([_vp, _vp, _i64, _i64, _i64, _i64, _int, _vp, _vp, _i64, _i64,
                              ctypes.c_float, _vp], _int),
    "pdd_sweep_plan_info": ([_vp, _vp], _int),
    "pdd_sweep_pattern_bytes": ([_vp, _i64], _i64),
    "pdd_sweep_execute_stage": ([_vp, _vp, _i64, _i64, _i64, _i64, _int, _vp, _vp, _i64, _i64,
                                 ctypes.c_float, _vp, _i64, _int, _vp], _int),
    "pdd_stream_create_cu_mask": ([_vp, _int, ctypes.POINTER(_vp)], _int),
    "pdd_stream_destroy": ([_vp], _int),
    "pdd_sweep_plan_set_input_max": ([_vp, _int], _int),
    "pdd_sweep_plan_destroy": ([_vp], _int),
    "pdd_global_stats": ([_vp, _i64, _i64, _i64, _vp, _vp], _int),
    "pdd_scale_rows": ([_vp, _i64, _i64, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _vp], _int),
    "pdd_masked_fill": ([_vp, _i64, _i64, _i64, _vp, _i64, _vp, _vp, _i64, _vp], _int),
    "pdd_smooth": ([_vp, _i64, _i64, _i64, _i64, _int, _vp, _vp, _i64, _vp], _int),
    "pdd_zdm_downsample": ([_vp, _int, _i64, _i64, _i64, _i64, _int, _vp, _i64, _vp], _int),
    "pdd_zdm_int_downsample": ([_vp, _int, _i64, _i64, _i64, _i64, _int, _int, _vp, _i64, _vp],
                               _int),
    "pdd_sweep_set_timing": ([_vp, _int], _int),
    "pdd_sweep_plan_create_grouped": ([_vp, _i64, _i64, _i64, _int, ctypes.POINTER(_vp)], _int),
    "pdd_sweep_execute_grouped": ([_vp, _vp, _i64, _i64, _int, _vp, _vp, _i64, _i64, _i64, _i64,
                                   _vp], _int),
    "pdd_sweep_execute_ds": ([_vp, _vp, _i64, _i64, _i64, _int, _vp, _vp, _i64, _i64, _i64, _i64,
                              _vp], _int),
    "pdd_subband_chain": ([_vp, _vp, _i64, _i64, _i64, _int, _vp, _vp, _vp, _vp, _i64, _i64,
                           _i64, _i64, _vp], _int),
    "pdd_sweep_kernel_ms": ([_vp, ctypes.POINTER(ctypes.c_float)], _int),
    "pdd_sweep_timing_read": ([_vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(_i64)], _int),
    "pdd_sp_chunk_stats": ([_vp, _i64, _i64, _i64, _i64, _vp, _vp, _vp], _int),
    "pdd_sp_search": ([_vp, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _i64, _i64, _vp, _vp, _i64,
                       _vp, _int, ctypes.c_float, _vp, _i64, _vp, _vp], _int),
    "pdd_psrfits_subints": ([_vp, _i64, _i64, _i64, _int, _i64, _i64, _vp, _i64, _i64, _int, _vp,
                             _i64, _vp], _int),
}


class PddStaleLibrary(PddLibraryMissing):
    pass


def open_library(path, check=True):
    """ctypes handle of the libpdd.so at `path` with every signature set.
    check: the library's compiled-in source digest must equal this tree's
    (a stale binary is refused, not used)."""
    h = ctypes.CDLL(path)
    for name, (argtypes, restype) in _SIGS.items():
        fn = getattr(h, name)
        fn.argtypes = argtypes
        fn.restype = restype
    if check and _digest.sources_present():
        got = h.pdd_source_digest().decode()
        want = _digest.source_digest()
        if got != want:
            raise PddStaleLibrary(
                "%s was built from other sources (digest %s, this tree %s): rebuild it with "
                "`python -c 'import __graft_entry__ as g; g.build()'`" % (path, got, want))
    return h


def lib():
    """Load (once) and return the ctypes handle of libpdd.so."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise PddLibraryMissing(
                "libpdd.so not found at %s: build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'`" % LIB_PATH)
        _lib = open_library(LIB_PATH, check=not _DEV_LIB)
    return _lib


def loaded_digest():
    """Source digest compiled into the loaded library."""
    return lib().pdd_source_digest().decode()


def check(status, what):
    if status != 0:
        msg = lib().pdd_last_error()
        raise PddError("%s failed (status %d): %s" % (what, status,
                                                      msg.decode() if msg else "?"))


def call(name, *args):
    check(getattr(lib(), name)(*args), name)


def ptr(t):
    """Device pointer of a CUDA tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise PddError("expected a device tensor, got one on %s" % t.device)
    return ctypes.c_void_p(t.data_ptr())


def stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def require_gpu():
    if not torch.cuda.is_available():
        raise PddError("pypulsar_amd needs a ROCm GPU (torch.cuda.is_available() is False); "
                       "there is no CPU fallback")
    lib()
