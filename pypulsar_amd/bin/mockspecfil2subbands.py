#!/usr/bin/env python
"""mockspecfil2subbands.py -- filterbank -> one PRESTO subband file per channel.

Drop-in for pypulsar's bin/mockspecfil2subbands.py (same -o/--outname option
and outputs): ``<outname>.sub.inf`` (writeInfoFile, mockspecfil2subbands.py:
40-129) and ``<outname>.subNNNN`` raw channel files, numbered in reverse
channel order when foff < 0 (:140-146).

The corner turn ([time, chan] -> [chan, time], :159-160) runs on the GPU
(pdd_corner_turn, raw dtype) over large blocks.  The reference's intended
Python-2 sample selection is kept by default: its loop starts at 1
(:155), so it writes the first (N//4096 - 1)*4096 spectra and then the
N % 4096 that follow -- N - 4096 spectra when N >= 4096 -- while the .inf
states N.  ``--all-samples`` writes all N instead.
"""
import optparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SAMPLES_PER_READ = 1024 * 4  # mockspecfil2subbands.py:20
BLOCK = SAMPLES_PER_READ * 64  # spectra per device corner turn


def _parse_rastr(rastr):
    """(h, m, s) strings of an HHMMSS.SSSS value (utils/coordconv.py:175-203)."""
    rastr = str(rastr)
    if float(rastr) == 0:
        return ("00", "00", "00")
    if rastr[0] == "+":
        rastr = rastr[1:]
    if "." in rastr:
        a, b = rastr.split(".", 1)
        b = "." + b
    else:
        a, b = rastr, ""
    a = a.zfill(6)
    return a[0:2], a[2:4], "%s%s" % (a[4:6], b)


def rastr_to_fmrastr(rastr):
    """HH:MM:SS.SSSS (utils/coordconv.py:145-155)."""
    return "%s:%s:%s" % _parse_rastr(rastr)


def decstr_to_fmdecstr(decstr):
    """+/-DD:MM:SS.SSSS (utils/coordconv.py:37-84)."""
    decl = float(str(decstr))
    if decl == 0:
        return "+00:00:00"
    sign = "+" if decl > 0 else "-"
    d = str(abs(decl))
    if "." in d:
        a, b = d.split(".", 1)
        b = "." + b
    else:
        a, b = d, ""
    a = a.zfill(6)
    return "%s%s:%s:%s%s" % (sign, a[0:2], a[2:4], a[4:6], b)


def write_inf(fb, outname, nsamples=None):
    """``<outname>.sub.inf`` exactly as writeInfoFile (mockspecfil2subbands.py:40-129)."""
    from pypulsar_amd.formats import sigproc
    h = fb.header
    base = "%s.sub" % outname
    tel = sigproc.ids_to_telescope.get(h.get("telescope_id"), "????")
    mach = sigproc.ids_to_machine.get(h.get("machine_id"), "????")
    if h["foff"] < 0:
        chanbw = -h["foff"]
        totalbw = chanbw * h["nchans"]
        lofreq = h["fch1"] - totalbw
    else:
        chanbw = h["foff"]
        totalbw = chanbw * h["nchans"]
        lofreq = h["fch1"]
    lines = [
        " Data file name without suffix          =  %s" % base,
        " Telescope used                         =  %s" % tel,
        " Instrument used                        =  %s" % mach,
        " Object being observed                  =  %s" % h.get("source_name", ""),
        " J2000 Right Ascension (hh:mm:ss.ssss)  =  %s" % rastr_to_fmrastr(h.get("src_raj", 0.0)),
        " J2000 Declination     (dd:mm:ss.ssss)  =  %s" % decstr_to_fmdecstr(h.get("src_dej", 0.0)),
        " Data observed by                       =  Unknown",
        " Epoch of observation (MJD)             =  %.15f" % h.get("tstart", 0.0),
        " Barycentered?           (1=yes, 0=no)  =  0",
        " Number of bins in the time series      =  %d" % (fb.number_of_samples if nsamples is None
                                                           else nsamples),
        " Width of each time series bin (sec)    =  %g" % h["tsamp"],
        " Any breaks in the data? (1=yes, 0=no)  =  0",
        " Type of observation (EM band)          =  Radio",
        " Beam diameter (arcsec)                 =  175",
        " Dispersion measure (cm-3 pc)           =  0",
        " Central freq of low channel (Mhz)      =  %f" % lofreq,
        " Total bandwidth (Mhz)                  =  %f" % totalbw,
        " Number of channels                     =  %d" % h["nchans"],
        " Channel bandwidth (Mhz)                =  %f" % chanbw,
        " Data analyzed by                       =  Patrick Lazarus",
        " Any additional notes:",
        "    Input filterbank file created from MockSpec data (AO)",
        "    using psrfits2fil, written by Julia Deneva (?)",
        "    Subbands and inf file created by mockspecfil2subbands.py",
        "    written by Patrick Lazarus, June 11, 2009",
    ]
    with open("%s.inf" % base, "w") as f:
        f.write("\n".join(lines) + "\n")


def samples_written(N, all_samples=False):
    """Number of leading spectra the reference's loop writes (:155-175)."""
    if all_samples:
        return N
    nblk = N // SAMPLES_PER_READ
    return max(0, nblk - 1) * SAMPLES_PER_READ + N % SAMPLES_PER_READ


def convert(infile, outname, all_samples=False, block=BLOCK):
    import torch
    from pypulsar_amd import _lib
    from pypulsar_amd._lib import call, ptr, stream_ptr
    from pypulsar_amd.formats import filterbank

    fb = filterbank.filterbank(infile)
    if fb.foff == 0:
        sys.stderr.write("Channel bandwidth is 0! Exiting...\n")
        return 1
    write_inf(fb, outname)
    C = fb.nchans
    order = range(C) if fb.foff > 0 else range(C - 1, -1, -1)
    names = ["%s.sub%04d" % (outname, k) for k in order]
    outs = [open(fn, "wb") for fn in names]
    np_dtype = np.dtype(fb.dtype)
    code = {1: _lib.U8, 2: _lib.U16, 4: _lib.F32}[np_dtype.itemsize]
    tdt = {1: torch.uint8, 2: torch.int16, 4: torch.float32}[np_dtype.itemsize]
    total = samples_written(fb.number_of_samples, all_samples)
    host = torch.empty((block, C), dtype=tdt, pin_memory=True)
    hview = host.numpy().view(np_dtype)
    done = 0
    while done < total:
        n = fb.read_block_into(done, hview[: min(block, total - done)])
        if n <= 0:
            break
        src = host[:n].to("cuda", non_blocking=True)
        dst = torch.empty((C, n), dtype=tdt, device="cuda")
        out_code = code if code != _lib.F32 else _lib.F32
        call("pdd_corner_turn", ptr(src), code, n, C, C, ptr(dst), out_code, n, stream_ptr())
        rows = dst.cpu().numpy().view(np_dtype)
        for j in range(C):
            rows[j].tofile(outs[j])
        done += n
    for f in outs:
        f.close()
    fb.close()
    return 0


def main(argv=None):
    parser = optparse.OptionParser(
        usage="%prog [options] infile",
        description="Convert filterbank data (from MockSpec data) to PRESTO subbands. "
                    "Each subband is one channel.")
    parser.add_option("-o", "--outname", dest="outname", type="string",
                      help="Output filename. Do not include extension.", default=None)
    parser.add_option("--all-samples", dest="all_samples", action="store_true", default=False,
                      help="Write all N spectra (the reference writes N - 4096).")
    options, args = parser.parse_args(argv)
    if len(args) == 0:
        parser.print_help()
        return 1
    if options.outname is None:
        sys.stderr.write("An outname must be provided. (Use -o/--outname on commandline).\n")
        return 1
    sys.stdout.write("Working...")
    rc = convert(args[0], options.outname, options.all_samples)
    sys.stdout.write("\rDone!       \n")
    sys.stdout.flush()
    return rc


if __name__ == "__main__":
    sys.exit(main())
