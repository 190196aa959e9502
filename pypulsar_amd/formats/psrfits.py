"""PSRFITS search-mode reader feeding the device ``Spectra`` (drop-in for
pypulsar's formats/psrfits.py).

Same names and behaviour as the reference: ``PsrfitsFile(fn)`` with
``filename``, ``fits``, ``specinfo``, ``header``, ``nbits``, ``nchan``,
``nsamp_per_subint``, ``nsubints``, ``freqs``/``frequencies``, ``tsamp``;
``read_subint``, ``get_weights``/``get_scales``/``get_offsets``,
``get_spectra``; ``SpectraInfo`` (psrfits.py:186-464) with its ``__str__``;
``unpack_4bit``, ``DATEOBS_to_MJD``, ``is_PSRFITS``, ``debug_mode``.

The data path is the device: ``get_spectra`` copies the needed SUBINT rows
(as stored, big-endian) to the GPU and one HIP kernel
(``pdd_psrfits_subints``) unpacks 4/8/16/32-bit samples, applies
``((data*scales)+offsets)*weights`` in float32 in the reference's order
(psrfits.py:103-106), transposes to ``[chan, time]``, cuts the requested
span and flips an ascending band (psrfits.py:140-183).  ``read_subint``
returns the same kernel's result as a host ``[nsamp, nchan]`` float32 array.

Differences, all where the reference cannot run here: the FITS container is
read by ``formats/fits.py`` (astropy absent); PRESTO's ``psr_utils`` and
``pyslalib`` are replaced by SECPERDAY = 86400 and the SLALIB sla_cldj
calendar formula (``_cldj``); ``get_spectra`` at the exact end of a file
reads only the subints it needs (the reference indexes one past the last
subint there and raises); multi-polarisation data (NPOL > 1 unsummed) is
rejected as in the reference's reshape.
"""
import os
import re
import warnings

import numpy as np

from . import fits as pyfits

SECPERDAY = 86400.0

date_obs_re = re.compile(r"^(?P<year>[0-9]{4})-(?P<month>[0-9]{2})-"
                         r"(?P<day>[0-9]{2})T(?P<hour>[0-9]{2}):"
                         r"(?P<min>[0-9]{2}):(?P<sec>[0-9]{2}"
                         r"(?:\.[0-9]+)?)$")

debug = True


def unpack_4bit(data):
    """Two 4-bit samples per byte, low nibble first (psrfits.py:37-50).
    Host helper; the device kernel decodes the same order."""
    data = np.asarray(data, dtype=np.uint8)
    return np.dstack([np.bitwise_and(15, data), data >> 4]).flatten()


def _cldj(iy, im, idd):
    """SLALIB sla_cldj: Gregorian calendar date -> Modified Julian Date
    (integer arithmetic with Fortran truncating division).  Returns
    (mjd, status)."""
    iy, im, idd = int(iy), int(im), int(idd)
    if iy < -4699:
        return 0.0, 1
    if im < 1 or im > 12:
        return 0.0, 2
    mtab = [31, 28 + (1 if (iy % 4 == 0 and (iy % 100 != 0 or iy % 400 == 0)) else 0),
            31, 30, 31, 30, 31, 31, 30, 31, 30, 31]
    status = 0 if 1 <= idd <= mtab[im - 1] else 3

    def tdiv(a, b):
        q = abs(a) // abs(b)
        return q if (a >= 0) == (b >= 0) else -q
    djm = (tdiv(1461 * (iy - tdiv(12 - im, 10) + 4712), 4)
           + tdiv(306 * ((im + 9) % 12) + 5, 10)
           - tdiv(3 * tdiv(iy - tdiv(12 - im, 10) + 4900, 100), 4)
           + idd - 2399904)
    return float(djm), status


def DATEOBS_to_MJD(dateobs):
    """DATE-OBS string -> (integer MJD, fractional day) (psrfits.py:563-575)."""
    m = date_obs_re.match(dateobs)
    mjd_fracday = (float(m.group("hour")) + (float(m.group("min")) +
                                             (float(m.group("sec")) / 60.0)) / 60.0) / 24.0
    mjd_day, err = _cldj(float(m.group("year")), float(m.group("month")), float(m.group("day")))
    return mjd_day, mjd_fracday


def is_PSRFITS(filename):
    """FITSTYPE == 'PSRFITS' and OBS_MODE == 'SEARCH' (psrfits.py:578-594)."""
    hdus = pyfits.open(filename, mode="readonly")
    primary = hdus["PRIMARY"].header
    try:
        ok = (primary["FITSTYPE"] == "PSRFITS") and (primary["OBS_MODE"] == "SEARCH")
    except KeyError:
        ok = False
    hdus.close()
    return ok


def debug_mode(mode=None):
    global debug
    if mode is None:
        return debug
    debug = bool(mode)


def _sexagesimal_to_deg(s, hours):
    """protractor.convert(s, 'hmsstr'|'dmsstr', 'deg') (utils/astro/protractor.py:19-80):
    [sign]DD:MM[:SS.S], the sign applying to the whole value; NaN if unparsable."""
    m = re.match(r"^(?P<sign>[-+])?(?P<a>\d{2}):(?P<b>\d{2})(?::(?P<c>\d{2}(?:.\d+)?))?$", str(s))
    if m is None:
        warnings.warn("Input is not a valid sexigesimal string: %s" % s)
        return float("nan")
    v = float(m.group("a")) + float(m.group("b")) / 60.0 + float(m.group("c") or 0) / 3600.0
    v = -v if m.group("sign") == "-" else v
    return v * 15.0 if hours else v


class SpectraInfo(object):
    """Header summary of one or more PSRFITS files (psrfits.py:186-464)."""

    def __init__(self, filenames):
        self.filenames = filenames
        self.num_files = len(filenames)
        self.N = 0
        self.user_poln = 0
        self.default_poln = 0
        self.start_MJD = np.empty(self.num_files)
        self.num_subint = np.empty(self.num_files)
        self.start_subint = np.empty(self.num_files)
        self.start_spec = np.empty(self.num_files)
        self.num_pad = np.empty(self.num_files)
        self.num_spec = np.empty(self.num_files)
        self.need_scale = False
        self.need_offset = False
        self.need_weight = False
        self.need_flipband = False

        for ii, fn in enumerate(filenames):
            if not is_PSRFITS(fn):
                raise ValueError("File '%s' does not appear to be PSRFITS!" % fn)
            hdus = pyfits.open(fn, mode="readonly")
            if ii == 0:
                self.hdu_names = [hdu.name for hdu in hdus]
            primary = hdus["PRIMARY"].header
            telescope = primary.get("TELESCOP", "")
            if telescope == "ARECIBO 305m":
                telescope = "Arecibo"
            if ii == 0:
                self.telescope = telescope
            elif telescope != self.telescope[0]:
                warnings.warn("'TELESCOP' values don't match for files 0 and %d!" % ii)
            self.observer = primary["OBSERVER"]
            self.source = primary["SRC_NAME"]
            self.frontend = primary["FRONTEND"]
            self.backend = primary["BACKEND"]
            self.project_id = primary["PROJID"]
            self.date_obs = primary["DATE-OBS"]
            self.poln_type = primary["FD_POLN"]
            self.ra_str = primary["RA"]
            self.dec_str = primary["DEC"]
            self.fctr = primary["OBSFREQ"]
            self.orig_num_chan = primary["OBSNCHAN"]
            self.orig_df = primary["OBSBW"]
            self.beam_FWHM = primary["BMIN"]
            self.chan_dm = primary.get("CHAN_DM", 0.0)
            self.start_MJD[ii] = primary["STT_IMJD"] + (primary["STT_SMJD"] +
                                                        primary["STT_OFFS"]) / SECPERDAY
            track = primary["TRK_MODE"] == "TRACK"
            if ii == 0:
                self.tracking = track
            elif track != self.tracking:
                warnings.warn("'TRK_MODE' values don't match for files 0 and %d" % ii)

            subint = hdus["SUBINT"].header
            self.dt = subint["TBIN"]
            self.num_channels = subint["NCHAN"]
            self.num_polns = subint["NPOL"]
            envval = os.getenv("PSRFITS_POLN")
            if envval is not None:
                ival = int(envval)
                if -1 < ival < self.num_polns:
                    print("Using polarisation %d (from 0-%d) from PSRFITS_POLN." %
                          (ival, self.num_polns - 1))
                    self.default_poln = ival
                    self.user_poln = 1
            self.poln_order = subint["POL_TYPE"]
            if subint["NCHNOFFS"] > 0:
                warnings.warn("first freq channel is not 0 in file %d" % ii)
            self.spectra_per_subint = subint["NSBLK"]
            self.bits_per_sample = subint["NBITS"]
            self.num_subint[ii] = subint["NAXIS2"]
            self.start_subint[ii] = subint["NSUBOFFS"]
            self.time_per_subint = self.dt * self.spectra_per_subint
            self.start_MJD[ii] += (self.time_per_subint * self.start_subint[ii]) / SECPERDAY
            MJDf = self.start_MJD[ii] - self.start_MJD[0]
            if MJDf < 0.0:
                raise ValueError("File %d seems to be from before file 0!" % ii)
            self.start_spec[ii] = (MJDf * SECPERDAY / self.dt + 0.5)

            sh = hdus["SUBINT"]
            names = sh.columns.names
            if "OFFS_SUB" not in names:
                warnings.warn("Can't find the 'OFFS_SUB' column!")
            else:
                col = names.index("OFFS_SUB")
                if ii == 0:
                    self.offs_sub_col = col
                elif self.offs_sub_col != col:
                    warnings.warn("'OFFS_SUB' column changes between files 0 and %d!" % ii)
            if "DATA" not in names:
                warnings.warn("Can't find the 'DATA' column!")
            else:
                col = names.index("DATA")
                if ii == 0:
                    self.data_col = col
                    self.FITS_typecode = sh.columns[self.data_col].format[-1]
                elif self.data_col != col:
                    warnings.warn("'DATA' column changes between files 0 and %d!" % ii)
            if "TEL_AZ" not in names:
                self.azimuth = 0.0
            elif ii == 0:
                self.tel_az_col = names.index("TEL_AZ")
                self.azimuth = sh.data[0]["TEL_AZ"]
            if "TEL_ZEN" not in names:
                self.zenith_ang = 0.0
            elif ii == 0:
                self.tel_zen_col = names.index("TEL_ZEN")
                self.zenith_ang = sh.data[0]["TEL_ZEN"]
            if "DAT_FREQ" not in names:
                warnings.warn("Can't find the channel freq column, 'DAT_FREQ'!")
            else:
                col = names.index("DAT_FREQ")
                freqs = np.atleast_1d(sh.data[0]["DAT_FREQ"]).astype(np.float64)
                if ii == 0:
                    self.freqs_col = col
                    self.df = freqs[1] - freqs[0]
                    self.lo_freq = freqs[0]
                    self.hi_freq = freqs[-1]
                    ftmp = freqs[1:] - freqs[:-1]
                    if np.any((ftmp - self.df)) > 1e-7:  # the reference's test, kept as is
                        warnings.warn("Channel spacing changes in file %d!" % ii)
                else:
                    if np.abs(self.df - (freqs[1] - freqs[0])) > 1e-7:
                        warnings.warn("Channel spacing between files 0 and %d!" % ii)
                    if np.abs(self.lo_freq - freqs[0]) > 1e-7:
                        warnings.warn("Low channel changes between files 0 and %d!" % ii)
                    if np.abs(self.hi_freq - freqs[-1]) > 1e-7:
                        warnings.warn("High channel changes between files 0 and %d!" % ii)
            for key, attr, unit in (("DAT_WTS", "dat_wts_col", 1.0),
                                    ("DAT_OFFS", "dat_offs_col", 0.0),
                                    ("DAT_SCL", "dat_scl_col", 1.0)):
                label = {"DAT_WTS": "weights", "DAT_OFFS": "offsets", "DAT_SCL": "scalings"}[key]
                if key not in names:
                    warnings.warn("Can't find the channel %s column, '%s'!" % (label, key))
                    continue
                col = names.index(key)
                if ii == 0:
                    setattr(self, attr, col)
                elif getattr(self, attr) != col:
                    warnings.warn("'%s' column changes between files 0 and %d!" % (key, ii))
                if np.any(np.atleast_1d(sh.data[0][key]) != unit):
                    if key == "DAT_WTS":
                        self.need_weight = True
                    elif key == "DAT_OFFS":
                        self.need_offset = True
                    else:
                        self.need_scale = True
            self.num_pad[ii] = 0
            self.num_spec[ii] = self.spectra_per_subint * self.num_subint[ii]
            if ii > 0 and self.start_spec[ii] > self.N:
                self.num_pad[ii - 1] = self.start_spec[ii] - self.N
                self.N += self.num_pad[ii - 1]
            self.N += self.num_spec[ii]

        self.ra2000 = _sexagesimal_to_deg(self.ra_str, hours=True)
        self.dec2000 = _sexagesimal_to_deg(self.dec_str, hours=False)
        self.summed_polns = self.poln_order in ("AA+BB", "INTEN")
        self.T = self.N * self.dt
        self.orig_df /= float(self.orig_num_chan)
        self.samples_per_spectra = self.num_polns * self.num_channels
        if self.bits_per_sample < 8:
            self.bytes_per_spectra = self.samples_per_spectra
        else:
            self.bytes_per_spectra = (self.bits_per_sample * self.samples_per_spectra) / 8
        self.samples_per_subint = self.samples_per_spectra * self.spectra_per_subint
        self.bytes_per_subint = self.bytes_per_spectra * self.spectra_per_subint
        if self.hi_freq < self.lo_freq:
            self.hi_freq, self.lo_freq = self.lo_freq, self.hi_freq
            self.df *= -1.0
            self.need_flipband = True
        self.BW = self.num_channels * self.df
        self.mjd = int(self.start_MJD[0])
        self.secs = (self.start_MJD[0] % 1) * SECPERDAY

    def __str__(self):
        """psrfits.py:466-557, same lines."""
        r = ["From the PSRFITS file '%s':" % self.filenames[0],
             "                       HDUs = %s" % ", ".join(self.hdu_names),
             "                  Telescope = %s" % self.telescope,
             "                   Observer = %s" % self.observer,
             "                Source Name = %s" % self.source,
             "                   Frontend = %s" % self.frontend,
             "                    Backend = %s" % self.backend,
             "                 Project ID = %s" % self.project_id,
             "            Obs Date String = %s" % self.date_obs]
        imjd, fmjd = DATEOBS_to_MJD(self.date_obs)
        mjdtmp = "%.14f" % fmjd
        r.append("  MJD start time (DATE-OBS) = %5d.%14s" % (imjd, mjdtmp[2:]))
        r.append("     MJD start time (STT_*) = %19.14f" % self.start_MJD[0])
        r.append("                   RA J2000 = %s" % self.ra_str)
        r.append("             RA J2000 (deg) = %-17.15g" % self.ra2000)
        r.append("                  Dec J2000 = %s" % self.dec_str)
        r.append("            Dec J2000 (deg) = %-17.15g" % self.dec2000)
        r.append("                  Tracking? = %s" % self.tracking)
        r.append("              Azimuth (deg) = %-.7g" % self.azimuth)
        r.append("           Zenith Ang (deg) = %-.7g" % self.zenith_ang)
        r.append("          Polarisation type = %s" % self.poln_type)
        if self.num_polns >= 2 and not self.summed_polns:
            numpolns = "%d" % self.num_polns
        elif self.summed_polns:
            numpolns = "2 (summed)"
        else:
            numpolns = "1"
        r.append("            Number of polns = %s" % numpolns)
        r.append("          Polarisation oder = %s" % self.poln_order)
        r.append("           Sample time (us) = %-17.15g" % (self.dt * 1e6))
        r.append("         Central freq (MHz) = %-17.15g" % self.fctr)
        r.append("          Low channel (MHz) = %-17.15g" % self.lo_freq)
        r.append("         High channel (MHz) = %-17.15g" % self.hi_freq)
        r.append("        Channel width (MHz) = %-17.15g" % self.df)
        r.append("         Number of channels = %d" % self.num_channels)
        if self.chan_dm != 0.0:
            r.append("   Orig Channel width (MHz) = %-17.15g" % self.orig_df)
            r.append("    Orig Number of channels = %d" % self.orig_num_chan)
            r.append("    DM used for chan dedisp = %-17.15g" % self.chan_dm)
        r.append("      Total Bandwidth (MHz) = %-17.15g" % self.BW)
        r.append("         Spectra per subint = %d" % self.spectra_per_subint)
        r.append("            Starting subint = %d" % self.start_subint[0])
        r.append("           Subints per file = %d" % self.num_subint[0])
        r.append("           Spectra per file = %d" % self.num_spec[0])
        r.append("        Time per file (sec) = %-.12g" % (self.num_spec[0] * self.dt))
        r.append("              FITS typecode = %s" % self.FITS_typecode)
        if debug:
            r.append("                DATA column = %d" % self.data_col)
            r.append("            bits per sample = %d" % self.bits_per_sample)
            if self.bits_per_sample < 8:
                spectmp = (self.bytes_per_spectra * self.bits_per_sample) / 8
                subtmp = (self.bytes_per_subint * self.bits_per_sample) / 8
            else:
                spectmp = self.bytes_per_spectra
                subtmp = self.bytes_per_subint
            r.append("          bytes per spectra = %d" % spectmp)
            r.append("        samples per spectra = %d" % self.samples_per_spectra)
            r.append("           bytes per subint = %d" % subtmp)
            r.append("         samples per subint = %d" % self.samples_per_subint)
            r.append("              Need scaling? = %s" % self.need_scale)
            r.append("              Need offsets? = %s" % self.need_offset)
            r.append("              Need weights? = %s" % self.need_weight)
            r.append("        Need band inverted? = %s" % self.need_flipband)
        return "\n".join(r)

    def __getitem__(self, key):
        return getattr(self, key)


class PsrfitsFile(object):
    def __init__(self, psrfitsfn):
        if not os.path.isfile(psrfitsfn):
            raise ValueError("ERROR: File does not exist!\n\t(%s)" % psrfitsfn)
        self.filename = psrfitsfn
        self.fits = pyfits.open(psrfitsfn, mode="readonly", memmap=True)
        self.specinfo = SpectraInfo([psrfitsfn])
        self.header = self.fits[0].header
        self.nbits = self.specinfo.bits_per_sample
        self.nchan = self.specinfo.num_channels
        self.nsamp_per_subint = self.specinfo.spectra_per_subint
        self.nsubints = int(self.specinfo.num_subint[0])
        self.freqs = np.atleast_1d(self.fits["SUBINT"].data[0]["DAT_FREQ"]).astype(np.float64)
        self.frequencies = self.freqs
        self.tsamp = self.specinfo.dt
        sub = self.fits["SUBINT"]
        names = sub.columns.names
        self._row_bytes = int(sub.header["NAXIS1"])
        self._data_off = sub.columns[names.index("DATA")].offset
        if self.nbits not in (4, 8, 16, 32):
            raise ValueError("PSRFITS nbits=%d is not supported (4, 8, 16, 32)" % self.nbits)
        npol = self.specinfo.num_polns
        if npol != 1 and not self.specinfo.summed_polns:
            raise ValueError("multi-polarisation (NPOL=%d) data cannot be reshaped to "
                             "(nsamp, nchan) (psrfits.py:104)" % npol)

    def get_weights(self, isub):
        return self.fits["SUBINT"].data[isub]["DAT_WTS"]

    def get_scales(self, isub):
        return self.fits["SUBINT"].data[isub]["DAT_SCL"]

    def get_offsets(self, isub):
        return self.fits["SUBINT"].data[isub]["DAT_OFFS"]

    def _wso(self, sub0, nsub, apply_weights=True, apply_scales=True, apply_offsets=True):
        """[nsub][3][nchan] float32: scales, offsets, weights (or 1, 0, 1)."""
        out = np.empty((nsub, 3, self.nchan), dtype=np.float32)
        for i in range(nsub):
            isub = sub0 + i
            out[i, 0] = np.asarray(self.get_scales(isub), dtype=np.float32)[:self.nchan] \
                if apply_scales else 1.0
            out[i, 1] = np.asarray(self.get_offsets(isub), dtype=np.float32)[:self.nchan] \
                if apply_offsets else 0.0
            out[i, 2] = np.asarray(self.get_weights(isub), dtype=np.float32)[:self.nchan] \
                if apply_weights else 1.0
        return out

    def _decode(self, sub0, nsub, s0, N, flip, apply_weights=True, apply_scales=True,
                apply_offsets=True):
        """Device [nchan, N] float32: samples s0 .. s0+N-1 of subints
        sub0 .. sub0+nsub-1 (pdd_psrfits_subints)."""
        import torch
        from .. import _lib
        from .._lib import call, ptr, stream_ptr
        _lib.require_gpu()
        if N == 0:
            return torch.empty((self.nchan, 0), dtype=torch.float32, device="cuda")
        rows = np.array(self.fits["SUBINT"].raw_rows(sub0, sub0 + nsub))  # host copy
        raw = torch.from_numpy(rows).pin_memory().cuda(non_blocking=True)
        wso = torch.from_numpy(self._wso(sub0, nsub, apply_weights, apply_scales,
                                         apply_offsets)).cuda()
        out = torch.empty((self.nchan, N), dtype=torch.float32, device="cuda")
        call("pdd_psrfits_subints", ptr(raw), nsub, self._row_bytes, self._data_off, self.nbits,
             self.nsamp_per_subint, self.nchan, ptr(wso), s0, N, int(bool(flip)), ptr(out),
             N, stream_ptr())
        return out

    def read_subint(self, isub, apply_weights=True, apply_scales=True, apply_offsets=True):
        """float32 [nsamp_per_subint, nchan] with scales, offsets and weights
        applied (psrfits.py:67-107), decoded on the device."""
        out = self._decode(isub, 1, 0, self.nsamp_per_subint, False, apply_weights,
                           apply_scales, apply_offsets)
        return out.t().contiguous().cpu().numpy()

    def get_spectra(self, startsamp, N):
        """Device Spectra of samples startsamp .. startsamp+N-1, high
        frequency first (psrfits.py:140-183)."""
        from .spectra import Spectra
        startsub = int(startsamp / self.nsamp_per_subint)
        skip = startsamp - startsub * self.nsamp_per_subint
        endsub = int((startsamp + N) / self.nsamp_per_subint)
        trunc = ((endsub + 1) * self.nsamp_per_subint) - (startsamp + N)
        if trunc < 0:
            raise ValueError("Number of bins to truncate is negative: %d" % trunc)
        # subints actually holding samples (the reference also reads endsub
        # when the span ends on a subint boundary; its samples are cut)
        last = min(endsub, (startsamp + N - 1) // self.nsamp_per_subint) if N > 0 else startsub
        if last >= self.nsubints:
            raise IndexError("samples up to %d requested, file has %d"
                             % (startsamp + N, self.nsubints * self.nsamp_per_subint))
        flip = not self.specinfo.need_flipband
        data = self._decode(startsub, last - startsub + 1, skip, N, flip)
        freqs = self.freqs[::-1] if flip else self.freqs
        return Spectra._from_device(np.array(freqs), self.tsamp, data,
                                    starttime=self.tsamp * startsamp)


def write_search_psrfits(fn, data, freqs, tbin, nbits, scales=None, offsets=None, weights=None,
                         primary=None, nsuboffs=0):
    """Write a single-polarisation search-mode PSRFITS file (test fixtures and
    mock data).  ``data``: [nsub, nsblk, nchan] samples in FILE channel order
    (uint8 0..15 for nbits 4 -- packed low nibble first, uint8 for 8, int16
    for 16, float32 for 32); ``freqs``: the DAT_FREQ column (either order);
    scales/offsets/weights: [nsub, nchan] (defaults 1, 0, 1)."""
    data = np.asarray(data)
    nsub, nsblk, nchan = data.shape
    if nbits == 4:
        flat = data.reshape(nsub, -1).astype(np.uint8)
        body = (flat[:, 0::2] & 15) | ((flat[:, 1::2] & 15) << 4)
        tform = "%dB" % body.shape[1]
    elif nbits == 8:
        body, tform = data.reshape(nsub, -1).astype(np.uint8), "%dB" % (nsblk * nchan)
    elif nbits == 16:
        body, tform = data.reshape(nsub, -1).astype(">i2"), "%dI" % (nsblk * nchan)
    elif nbits == 32:
        body, tform = data.reshape(nsub, -1).astype(">f4"), "%dE" % (nsblk * nchan)
    else:
        raise ValueError("nbits must be 4, 8, 16 or 32")
    ones = np.ones((nsub, nchan), dtype=np.float32)
    scales = ones if scales is None else np.asarray(scales, dtype=np.float32)
    offsets = 0 * ones if offsets is None else np.asarray(offsets, dtype=np.float32)
    weights = ones if weights is None else np.asarray(weights, dtype=np.float32)
    freqs = np.asarray(freqs, dtype=np.float64)
    cols = [("TSUBINT", "1D"), ("OFFS_SUB", "1D"), ("TEL_AZ", "1E"), ("TEL_ZEN", "1E"),
            ("DAT_FREQ", "%dD" % nchan), ("DAT_WTS", "%dE" % nchan), ("DAT_OFFS", "%dE" % nchan),
            ("DAT_SCL", "%dE" % nchan), ("DATA", tform)]
    rows = {
        "TSUBINT": np.full(nsub, nsblk * tbin), "OFFS_SUB": (np.arange(nsub) + 0.5) * nsblk * tbin,
        "TEL_AZ": np.full(nsub, 123.5, dtype=np.float32),
        "TEL_ZEN": np.full(nsub, 21.25, dtype=np.float32),
        "DAT_FREQ": np.tile(freqs, (nsub, 1)), "DAT_WTS": weights, "DAT_OFFS": offsets,
        "DAT_SCL": scales, "DATA": body,
    }
    p = [("FITSTYPE", "PSRFITS"), ("OBS_MODE", "SEARCH"), ("TELESCOP", "GBT"),
         ("OBSERVER", "pdd"), ("SRC_NAME", "J0000+0000"), ("FRONTEND", "Rcvr1_2"),
         ("BACKEND", "GUPPI"), ("PROJID", "TEST"), ("DATE-OBS", "2020-01-02T03:04:05.500"),
         ("FD_POLN", "LIN"), ("RA", "12:34:56.7"), ("DEC", "-01:23:45.6"),
         ("OBSFREQ", float(np.mean(freqs))), ("OBSNCHAN", nchan),
         ("OBSBW", float(abs(freqs[-1] - freqs[0]) * nchan / max(nchan - 1, 1))),
         ("BMIN", 0.15), ("CHAN_DM", 0.0), ("STT_IMJD", 58850), ("STT_SMJD", 11045),
         ("STT_OFFS", 0.5), ("TRK_MODE", "TRACK")]
    if primary:
        d = dict(p)
        d.update(primary)
        p = list(d.items())
    sub = [("TBIN", float(tbin)), ("NCHAN", nchan), ("NPOL", 1), ("POL_TYPE", "AA+BB"),
           ("NCHNOFFS", 0), ("NSBLK", nsblk), ("NBITS", nbits), ("NSUBOFFS", nsuboffs)]
    pyfits.write(fn, p, [("SUBINT", sub, cols, rows)])
