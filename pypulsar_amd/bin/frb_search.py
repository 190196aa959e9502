#!/usr/bin/env python
"""frb_search.py -- streaming single-pulse search of a SIGPROC filterbank.

New (the reference has no search; BASELINE config 5 plus its consumer):
blocks of spectra are read into rotating pinned host buffers
(filterbank.read_block_into), copied to the GPU on a copy stream, zero-DM
filtered (bin/zero_dm_filter.py:30-39, float mode), downsampled
(spectra.py:329-351), swept over a uniform DM grid (per-DM
Spectra.dedisperse + channel sum, spectra.py:229-260) and boxcar-searched
(pypulsar_amd.search; boxcar of pulse.py:217-241); only candidates come back
to the host.  The candidates equal those of a one-shot search of the whole
file's DM-time plane.  Output: PRESTO-style ``.singlepulse`` text.

    python -m pypulsar_amd.bin.frb_search --lodm 0 --hidm 1000 --numdms 2048 \\
        --downsamp 2 --threshold 7 -o obs.singlepulse obs.fil
"""
import optparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def _chunks(fb, block, nbuf=4, start_block=0):
    """Pinned [n, nchans] host chunks of the file from block ``start_block``
    on, in rotation (a buffer is reused nbuf chunks later, after its
    asynchronous copy has completed: StreamingSweep keeps at most 2 chunks in
    flight)."""
    import torch
    tdt = {np.dtype(np.uint8): torch.uint8, np.dtype(np.uint16): torch.int16,
           np.dtype(np.float32): torch.float32}[np.dtype(fb.dtype)]
    bufs = [torch.empty((block, fb.nchans), dtype=tdt, pin_memory=True) for _ in range(nbuf)]
    done, i = int(start_block) * block, 0
    while done < fb.number_of_samples:
        h = bufs[i % nbuf]
        n = fb.read_block_into(done, h.numpy().view(np.dtype(fb.dtype))[:block])
        if n <= 0:
            break
        yield h[:n]
        done += n
        i += 1


def search_file(infile, dms, downsamp=2, block=1 << 18, zero_dm=True, threshold=6.0,
                widths=None, detrendlen=1024, debug=False):
    import torch
    from pypulsar_amd.formats import filterbank
    from pypulsar_amd.search import DEFAULT_WIDTHS, StreamingSearch, merge

    fb = filterbank.filterbank(infile)
    if np.dtype(fb.dtype) == np.uint16:
        raise ValueError("16-bit filterbanks: convert to 8 or 32 bits first")
    tdt = torch.uint8 if np.dtype(fb.dtype) == np.uint8 else torch.float32
    ss = StreamingSearch(dms, fb.freqs, fb.tsamp, block=block, downsamp=downsamp,
                         zero_dm=zero_dm, dtype=tdt, threshold=threshold,
                         widths=widths or DEFAULT_WIDTHS, detrendlen=detrendlen)
    parts = []  # candidate times are relative to the file start
    for i, c in enumerate(ss(_chunks(fb, block))):
        parts.append(c)
        if debug:
            sys.stderr.write("\rblock %d: %d candidates" % (i, sum(len(p) for p in parts)))
    if debug:
        sys.stderr.write("\n")
    ss.close()
    fb.close()
    return merge(parts)


def main(argv=None):
    parser = optparse.OptionParser(prog="frb_search.py", usage="%prog [OPTIONS] INFILE",
                                   description="Streaming dedispersion + single-pulse search "
                                               "of a SIGPROC filterbank on the GPU.")
    parser.add_option("--lodm", type="float", default=0.0, help="Lowest DM (pc/cc).")
    parser.add_option("--hidm", type="float", default=1000.0, help="Highest DM (pc/cc).")
    parser.add_option("--numdms", type="int", default=1024, help="Number of DM trials.")
    parser.add_option("--downsamp", type="int", default=2,
                      help="Downsampling factor (divides 64). (Default: 2)")
    parser.add_option("--block", type="int", default=1 << 18,
                      help="Spectra per streamed block. (Default: 262144)")
    parser.add_option("--no-zero-dm", dest="zero_dm", action="store_false", default=True,
                      help="Skip the zero-DM filter.")
    parser.add_option("-t", "--threshold", type="float", default=6.0,
                      help="Candidate S/N threshold. (Default: 6)")
    parser.add_option("-m", "--maxwidth", type="int", default=150,
                      help="Largest boxcar width in downsampled samples (<= 1025).")
    parser.add_option("-o", "--outname", default=None,
                      help="Output .singlepulse file (default: INFILE with .singlepulse).")
    parser.add_option("-d", "--debug", action="store_true", default=False)
    options, args = parser.parse_args(argv)
    if len(args) != 1:
        parser.error("one input filterbank expected")
    from pypulsar_amd.search import DEFAULT_WIDTHS, write_singlepulse
    widths = tuple(w for w in DEFAULT_WIDTHS if w <= options.maxwidth) or (1,)
    dms = np.linspace(options.lodm, options.hidm, options.numdms)
    cands = search_file(args[0], dms, options.downsamp, options.block, options.zero_dm,
                        options.threshold, widths, debug=options.debug)
    out = options.outname or os.path.splitext(args[0])[0] + ".singlepulse"
    write_singlepulse(cands, out)
    print("%d candidates -> %s" % (len(cands), out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
