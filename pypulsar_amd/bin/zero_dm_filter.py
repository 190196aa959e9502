#!/usr/bin/env python
"""zero_dm_filter.py -- Zero-DM filter a SIGPROC filterbank on the GPU.

Drop-in for pypulsar's bin/zero_dm_filter.py (same options: -o/--outname,
-d/--debug, one input file).  Per spectrum the channel mean is subtracted
(bin/zero_dm_filter.py:30-39): integer data use the float64 mean rounded
half-to-even and cast to the data type, so the subtraction wraps modulo
2**nbits; float32 data stay float32.  The header is copied keyword by keyword
(zero_dm_filter.py:21-27).

The reference processes one spectrum per Python iteration and then crashes
writing a list (zero_dm_filter.py:48-50); this writes what it intended.
Blocks of spectra are read straight into a pinned host buffer, filtered by
pdd_zero_dm on the device and written back in file order.
"""
import optparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

BLOCK = 1 << 16  # spectra per device round trip


def filter_file(infile, outname, block=BLOCK, debug=False):
    import torch
    from pypulsar_amd import zero_dm as zd
    from pypulsar_amd.formats import filterbank, sigproc

    fb = filterbank.filterbank(infile)
    nchan = fb.nchans
    np_dtype = np.dtype(fb.dtype)
    tdt = {np.dtype(np.uint8): torch.uint8, np.dtype(np.uint16): torch.int16,
           np.dtype(np.float32): torch.float32}[np_dtype]
    host = torch.empty((block, nchan), dtype=tdt, pin_memory=True)
    hview = host.numpy().view(np_dtype)
    with open(outname, "wb") as out:
        sigproc.write_header(out, fb.header_params, fb.header)
        done = 0
        while done < fb.number_of_samples:
            n = fb.read_block_into(done, hview[: min(block, fb.number_of_samples - done)])
            if n <= 0:
                break
            if np_dtype == np.uint16:
                res = zd.zero_dm(hview[:n].copy(), layout="time")
            else:
                dev = host[:n].to("cuda", non_blocking=True)
                res = zd.zero_dm(dev, layout="time").cpu().numpy()
            np.ascontiguousarray(res).view(np_dtype).tofile(out)
            done += n
            if debug:
                sys.stderr.write("\r%d / %d spectra" % (done, fb.number_of_samples))
    fb.close()
    if debug:
        sys.stderr.write("\n")
    return done


def main(argv=None):
    parser = optparse.OptionParser(usage="%prog [options] infile",
                                   description="Perfom Zero-DM Filter on filterbank file.")
    parser.add_option("-o", "--outname", dest="outname", type="string",
                      help="Output filename.", default=None)
    parser.add_option("-d", "--debug", dest="debug", action="store_true",
                      help="Print useful debugging information. "
                           "(Default: Don't print debug info.)", default=False)
    options, args = parser.parse_args(argv)
    if len(args) == 0:
        parser.print_help()
        return 1
    if len(args) != 1:
        sys.stderr.write("Only one input file must be provided!\n")
        return 1
    if options.outname is None:
        sys.stderr.write("An outname must be provided. (Use -o/--outname on command line).\n")
        return 1
    sys.stdout.write("Working...")
    sys.stdout.flush()
    filter_file(args[-1], options.outname, debug=options.debug)
    sys.stdout.write("\rDone!" + " " * 50 + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
