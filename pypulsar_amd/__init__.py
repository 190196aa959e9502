"""pypulsar_amd — MI355X-native incoherent-dedispersion engine.

Drop-in for the dedispersion hot path of pypulsar (emilieparent/pypulsar):
``formats/spectra.py``'s ``Spectra`` (dedisperse, subband, downsample,
shift_channels, trim), the zero-DM filter of ``bin/zero_dm_filter.py``, and a
new batched DM-trial sweep over ``utils/DDplan2b.py`` grids.  Compute runs in
hand-written HIP kernels for gfx950 (libpdd.so, C ABI in include/pdd.h);
there is no CPU fallback.
"""
__version__ = "0.1.0"

__all__ = ["formats", "utils", "delays", "sweep", "zero_dm"]
