#!/usr/bin/env python
"""waterfaller.py -- waterfall plot of a single pulse in SIGPROC filterbank data.

Drop-in for pypulsar's bin/waterfaller.py (same options and pipeline,
waterfaller.py:51-208) on the device ``Spectra``: read (filterbank.get_spectra)
-> subband(nsub, subdm, padval='mean') -> dedisperse(dm, padval='mean',
trim=True) -> downsample -> scaled -> smooth -> plot, with every step a HIP
kernel and only the final 2-D image and summed series copied to the host.

Differences from the reference, all where it cannot run:
  * ``--mask`` reads the rfifind ``.mask`` file with
    pypulsar_amd.formats.rfifind (a restatement of PRESTO's format; PRESTO is
    absent) and masks on the device (Spectra.masked, 'median-mid80');
    ``.fits`` input goes through pypulsar_amd.formats.psrfits (device decode);
  * with dm == 0 the reference's ``dmtime`` is unbound (waterfaller.py:193-196):
    here it is 0;
  * ``-n/--nbins`` is honoured when no duration is given (the reference
    always passes duration + dmtime);
  * ``--outfile FILE`` saves the figure (a headless box has no window);
    without it the figure is shown as in the reference.
"""
import optparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SWEEP_STYLES = ["r-", "b-", "g-", "m-", "c-"]


def open_data_file(fn):
    from pypulsar_amd.formats import filterbank
    if fn.endswith(".fil"):
        return filterbank.filterbank(fn)
    if fn.endswith(".fits"):
        from pypulsar_amd.formats import psrfits
        return psrfits.PsrfitsFile(fn)
    raise ValueError("Cannot recognize data file type from extension. "
                     "(Only '.fits' and '.fil' are supported.)")


def get_data(rawdatafile, start, duration=None, nbins=None, mask=None):
    """Spectra of the requested span (waterfaller.py:67-100)."""
    start_bin = int(np.round(start / rawdatafile.tsamp))
    if nbins is None:
        if duration is None:
            raise ValueError("At least one of 'duration' and 'nbins' must be provided!")
        nbins = int(np.round(duration / rawdatafile.tsamp))
    data = rawdatafile.get_spectra(start_bin, nbins)
    if mask is not None:
        from pypulsar_amd.formats import rfifind
        rfimask = mask if isinstance(mask, rfifind.rfifind) else rfifind.rfifind(mask)
        datamask = rfifind.get_mask(rfimask, start_bin, nbins)
        data = data.masked(datamask, maskval="median-mid80")
    return data


def prepare_data(data, smooth=1, downsamp=1, dm=0, nsub=None, subdm=None, scaleindep=False,
                 noscale=False):
    """waterfaller.py:103-127, on the device."""
    if nsub is None:
        nsub = data.numchans
    if subdm is None:
        subdm = dm
    data.subband(nsub, subdm, padval="mean")
    if dm:
        data.dedisperse(dm, padval="mean", trim=True)
    if downsamp > 1:
        data.downsample(downsamp)
    if not noscale:
        data = data.scaled(scaleindep)
    if smooth > 1:
        data.smooth(smooth, padval="mean")
    return data


def plot(data, cmap="gist_yarg", show_cb=False, sweep_dms=None, sweep_posns=None):
    """waterfaller.py:130-186: the image and the summed series (channel sum
    computed on the device, waterfaller.py:140)."""
    import matplotlib.pyplot as plt
    from pypulsar_amd.delays import delay_from_DM
    sweep_dms = sweep_dms or []
    img = data.data
    series = data.sum_channels().cpu().numpy()
    freqs = np.asarray(data.freqs)
    ax = plt.axes((0.15, 0.15, 0.8, 0.7))
    plt.imshow(img, aspect="auto", cmap=plt.get_cmap(cmap), interpolation="nearest", origin="upper",
               extent=(data.starttime, data.starttime + data.numspectra * data.dt,
                       freqs.min(), freqs.max()))
    if show_cb:
        cb = plt.colorbar()
        cb.set_label("Scaled signal intensity (arbitrary units)")
    plt.axis("tight")
    for ii, sweep_dm in enumerate(sweep_dms):
        delays = delay_from_DM(sweep_dm - data.dm, freqs)
        delays -= delays.min()
        if not sweep_posns:
            sweep_posn = 0.0
        elif len(sweep_posns) == 1:
            sweep_posn = sweep_posns[0]
        else:
            sweep_posn = sweep_posns[ii]
        sweepstart = data.dt * data.numspectra * sweep_posn + data.starttime
        plt.plot(delays + sweepstart, freqs, SWEEP_STYLES[ii % len(SWEEP_STYLES)], lw=4, alpha=0.5)
    plt.xlabel("Time")
    plt.ylabel("Observing frequency (MHz)")
    sumax = plt.axes((0.15, 0.85, 0.8, 0.1), sharex=ax)
    times = np.arange(0, data.numspectra) * data.dt + data.starttime
    plt.plot(times, series, "k-")
    plt.setp(sumax.get_xticklabels() + sumax.get_yticklabels(), visible=False)
    plt.ylabel("Intensity")
    plt.ticklabel_format(style="plain", useOffset=False)
    plt.axis("tight")
    return sumax, ax


def run(fn, options):
    from pypulsar_amd.delays import delay_from_DM
    rawdatafile = open_data_file(fn)
    dmtime = float(delay_from_DM(options.dm, np.min(rawdatafile.freqs))) if options.dm else 0.0
    if options.duration is not None:
        data = get_data(rawdatafile, start=options.start, duration=options.duration + dmtime,
                        mask=options.maskfile)
    else:
        nb = options.nbins + int(np.round(dmtime / rawdatafile.tsamp))
        data = get_data(rawdatafile, start=options.start, nbins=nb, mask=options.maskfile)
    data = prepare_data(data, options.width_bins, options.downsamp, options.dm, options.nsub,
                        options.subdm, options.scaleindep)
    return data


def main(argv=None):
    parser = optparse.OptionParser(prog="waterfaller.py", usage="%prog [OPTIONS] INFILE",
                                   description="Create a waterfall plot to show the frequency "
                                               "sweep of a single pulse in SIGPROC filterbank data.")
    parser.add_option("--subdm", dest="subdm", type="float", default=None,
                      help="DM to use when subbanding. (Default: same as --dm)")
    parser.add_option("-s", "--nsub", dest="nsub", type="int", default=None,
                      help="Number of subbands to use. Must be a factor of number of channels. "
                           "(Default: number of channels)")
    parser.add_option("-d", "--dm", dest="dm", type="float", default=0.0,
                      help="DM to use when dedispersing data for plot. (Default: 0 pc/cm^3)")
    parser.add_option("-T", "--start-time", dest="start", type="float",
                      help="Time into observation (in seconds) at which to start plot.")
    parser.add_option("-t", "--duration", dest="duration", type="float",
                      help="Duration (in seconds) of plot.")
    parser.add_option("-n", "--nbins", dest="nbins", type="int",
                      help="Number of time bins to plot.")
    parser.add_option("--width-bins", dest="width_bins", type="int", default=1,
                      help="Smooth each channel/subband with a boxcar this many bins wide.")
    parser.add_option("--sweep-dm", dest="sweep_dms", type="float", action="append", default=[],
                      help="Show the frequency sweep using this DM.")
    parser.add_option("--sweep-posn", dest="sweep_posns", type="float", action="append",
                      default=None, help="Show the frequency sweep at this position (0..1).")
    parser.add_option("--downsamp", dest="downsamp", type="int", default=1,
                      help="Factor to downsample data by. (Default: 1).")
    parser.add_option("--mask", dest="maskfile", type="string", default=None,
                      help="Mask file produced by rfifind. (Default: No Mask).")
    parser.add_option("--scaleindep", dest="scaleindep", action="store_true", default=False,
                      help="If this flag is set scale each channel independently.")
    parser.add_option("--show-colour-bar", dest="show_cb", action="store_true", default=False,
                      help="If this flag is set show a colour bar.")
    parser.add_option("--colour-map", dest="cmap", default="gist_yarg",
                      help="The name of a valid matplotlib colour map.")
    parser.add_option("--outfile", dest="outfile", default=None,
                      help="Save the figure to this file instead of showing it.")
    options, args = parser.parse_args(argv)
    if options.start is None:
        raise ValueError("Start time (-T/--start-time) must be given on command line!")
    if options.duration is None and options.nbins is None:
        raise ValueError("One of duration (-t/--duration) and num bins (-n/--nbins) "
                         "must be given on command line!")
    if options.subdm is None:
        options.subdm = options.dm
    data = run(args[0], options)
    import matplotlib
    if options.outfile or not os.environ.get("DISPLAY"):
        matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    fig = plt.figure()
    plot(data, options.cmap, options.show_cb, options.sweep_dms, options.sweep_posns)
    if options.outfile:
        fig.savefig(options.outfile)
    else:
        plt.show()
    return 0


if __name__ == "__main__":
    sys.exit(main())
