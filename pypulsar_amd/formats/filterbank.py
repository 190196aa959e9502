"""SIGPROC filterbank reader feeding the device ``Spectra`` (drop-in for
pypulsar's formats/filterbank.py:19-157).

Same class, attributes and methods as the reference: ``filterbank(fn)`` reads
the header on construction (``read_header``, filterbank.py:45-68) and the
channel frequencies ``fch1 + foff*arange(nchans)`` (filterbank.py:77-87);
``header`` / ``header_params`` / ``number_of_samples`` / ``dtype`` /
``frequencies`` / ``freqs`` / ``is_hifreq_first``; header keywords as
attributes (``fb.tsamp``, ``fb.nchans``; filterbank.py:36-37);
``read_sample``, ``read_all_samples``, ``read_Nsamples``, ``seek_to_*`` and
``get_spectra(startsamp, N)``, which returns a device ``Spectra``
(the ``[N, C]`` block is corner-turned on the GPU).

Python-2 semantics the reference relies on are kept: the sample count and
the seek offset use integer byte counts (``nbits/8`` was integer division,
filterbank.py:65,68,134).

New for the streaming pipeline: ``read_block_into(startsamp, out)`` reads
samples straight into a caller-owned (e.g. pinned) host buffer.
"""
import os
import warnings

import numpy as np

from . import sigproc


class filterbank(object):
    def __init__(self, filfn):
        self.filename = filfn
        self.already_read_header = False
        self.header_params = []
        self.header = {}
        self.header_size = None
        self.data_size = None
        self.number_of_samples = None
        self.dtype = None
        self.filfile = None
        if not os.path.isfile(filfn):
            raise ValueError("ERROR: File does not exist!\n\t(%s)" % filfn)
        self.filfile = open(filfn, "rb")
        self.read_header()
        self.compute_frequencies()

    def __getattr__(self, name):
        # header keywords as attributes (filterbank.py:36-37)
        header = self.__dict__.get("header")
        if header is not None and name in header:
            return header[name]
        raise AttributeError(name)

    def close(self):
        if self.filfile is not None and not self.filfile.closed:
            self.filfile.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def read_header(self):
        if self.already_read_header:
            return
        self.already_read_header = True
        self.seek_to_header_start()
        self.header, self.header_params, self.header_size = sigproc.read_header(self.filfile)
        nbits = self.header["nbits"]
        if nbits not in (8, 16, 32):
            raise ValueError("unsupported nbits %d (8, 16 or 32)" % nbits)
        self.dtype = "float32" if nbits == 32 else "uint%d" % nbits
        self.data_size = os.stat(self.filename).st_size - self.header_size
        bytes_per_sample = self.header["nchans"] * (nbits // 8)
        if self.data_size % bytes_per_sample:
            warnings.warn("Not an integer number of samples in file.")
        self.number_of_samples = self.data_size // bytes_per_sample

    def print_header(self):
        self.read_header()
        for param in self.header_params:
            print("%s: %s" % (param, self.header[param]))

    def compute_frequencies(self):
        self.read_header()
        self.frequencies = self.header["fch1"] + self.header["foff"] * np.arange(self.header["nchans"])
        self.freqs = self.frequencies
        self.is_hifreq_first = (self.header["foff"] < 0)

    @property
    def bytes_per_spectrum(self):
        return self.header["nchans"] * (self.header["nbits"] // 8)

    def read_sample(self):
        self.read_header()
        return np.fromfile(self.filfile, dtype=self.dtype, count=self.header["nchans"])

    def read_all_samples(self):
        self.seek_to_data_start()
        return np.fromfile(self.filfile, dtype=self.dtype)

    def read_Nsamples(self, N):
        self.read_header()
        return np.fromfile(self.filfile, dtype=self.dtype, count=self.header["nchans"] * N)

    def seek_to_header_start(self):
        self.filfile.seek(0)

    def seek_to_data_start(self):
        self.read_header()
        self.filfile.seek(self.header_size)

    def seek_to_sample(self, sampnum):
        self.read_header()
        self.filfile.seek(self.header_size + self.bytes_per_spectrum * int(sampnum))

    def seek_to_position(self, posn):
        self.filfile.seek(posn)

    def get_spectra(self, startsamp, N):
        """[nchans, N] device Spectra of samples startsamp .. startsamp+N-1
        (filterbank.py:143-157): the [N, nchans] block is handed over as its
        transpose, which Spectra corner-turns on the GPU."""
        from .spectra import Spectra
        self.seek_to_sample(startsamp)
        data = self.read_Nsamples(N)
        data.shape = (N, self.header["nchans"])
        return Spectra(self.frequencies, self.header["tsamp"], data.T,
                       starttime=self.header["tsamp"] * startsamp, dm=0)

    def read_block_into(self, startsamp, out):
        """Read samples [startsamp, startsamp + len(out)) into ``out``, a
        C-contiguous host array (numpy, or a pinned torch tensor's .numpy())
        of shape [n, nchans] and the file's dtype; returns the number of whole
        spectra read (fewer at the end of the file).  A non-contiguous
        ``out`` is refused (ValueError): the bytes would land in a temporary
        copy, not in ``out``."""
        if not isinstance(out, np.ndarray) or not out.flags["C_CONTIGUOUS"]:
            raise ValueError("read_block_into: out must be a C-contiguous numpy array")
        if out.ndim != 2 or out.shape[1] != self.header["nchans"] or out.dtype != self.dtype:
            raise ValueError("read_block_into: out must be [n, %d] of %s, not %s of %s"
                             % (self.header["nchans"], self.dtype, out.shape, out.dtype))
        self.seek_to_sample(startsamp)
        buf = memoryview(out.view(np.uint8).reshape(-1))
        got = self.filfile.readinto(buf)
        return got // self.bytes_per_spectrum


def write_filterbank(fn, header_params, header, data):
    """Write a filterbank file: the header keywords in order, then ``data``
    ([nspec, nchans], dtype matching header nbits) in file order."""
    with open(fn, "wb") as f:
        sigproc.write_header(f, header_params, header)
        np.ascontiguousarray(data).tofile(f)
