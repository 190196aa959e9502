"""SIGPROC filterbank header codec (host side).

The reference reads and writes filterbank headers through PRESTO's
``sigproc`` module (``read_hdr_val`` at formats/filterbank.py:53,
``addto_hdr`` at bin/zero_dm_filter.py:26, ``ids_to_telescope`` /
``ids_to_machine`` at bin/mockspecfil2subbands.py:52-63).  PRESTO is not
vendored and not installed here, so this module restates the public SIGPROC
header format it implements:

  * every keyword is a length-prefixed string: int32 length (little endian)
    followed by that many ASCII bytes;
  * the keyword is followed by its value: int32 for integer keywords, float64
    for floating-point keywords, a length-prefixed string for string
    keywords, one signed byte for ``signed``, nothing for the
    HEADER_START / HEADER_END / FREQUENCY_START / FREQUENCY_END flags.

Parity with PRESTO's module itself is unpinned (no reference test or fixture
holds a header); the codec is checked by round trips and by hand-built byte
strings in tests/test_filterbank.py.
"""
import struct

INT_KEYS = ("telescope_id", "machine_id", "data_type", "barycentric", "pulsarcentric",
            "nbits", "nsamples", "nchans", "nifs", "nbeams", "ibeam")
DOUBLE_KEYS = ("tstart", "tsamp", "fch1", "foff", "refdm", "az_start", "za_start",
               "src_raj", "src_dej", "period", "fchannel", "refrf")
STRING_KEYS = ("source_name", "rawdatafile")
BYTE_KEYS = ("signed",)
FLAG_KEYS = ("HEADER_START", "HEADER_END", "FREQUENCY_START", "FREQUENCY_END")

# SIGPROC telescope / backend identifiers (used by the .inf writer of
# bin/mockspecfil2subbands.py:51-63)
ids_to_telescope = {0: "Fake", 1: "Arecibo", 2: "Ooty", 3: "Nancay", 4: "Parkes",
                    5: "Jodrell", 6: "GBT", 7: "GMRT", 8: "Effelsberg", 9: "ATA",
                    10: "UTR-2", 11: "LOFAR", 12: "FR606", 20: "CHIME", 64: "MeerKAT"}
ids_to_machine = {0: "FAKE", 1: "PSPM", 2: "WAPP", 3: "AOFTM", 4: "BCPM1", 5: "OOTY",
                  6: "SCAMP", 7: "GBT Pulsar Spigot", 8: "PFFTS", 9: "GUPPI",
                  10: "CHIME", 11: "PUPPI"}
telescope_to_id = dict((v, k) for k, v in ids_to_telescope.items())
machine_to_id = dict((v, k) for k, v in ids_to_machine.items())


def _read_string(f):
    raw = f.read(4)
    if len(raw) < 4:
        raise EOFError("truncated SIGPROC header")
    n = struct.unpack("<i", raw)[0]
    if n < 0 or n > 4096:
        raise ValueError("not a SIGPROC header (keyword length %d)" % n)
    s = f.read(n)
    if len(s) < n:
        raise EOFError("truncated SIGPROC header")
    return s.decode("ascii")


def _pack_string(s):
    b = s.encode("ascii")
    return struct.pack("<i", len(b)) + b


def read_hdr_val(f):
    """Read one (keyword, value) pair from the open binary file ``f``
    (the role of PRESTO's sigproc.read_hdr_val, formats/filterbank.py:53)."""
    key = _read_string(f)
    if key in FLAG_KEYS:
        return key, None
    if key in INT_KEYS:
        return key, struct.unpack("<i", f.read(4))[0]
    if key in DOUBLE_KEYS:
        return key, struct.unpack("<d", f.read(8))[0]
    if key in STRING_KEYS:
        return key, _read_string(f)
    if key in BYTE_KEYS:
        return key, struct.unpack("<b", f.read(1))[0]
    raise ValueError("unknown SIGPROC header keyword %r" % key)


def addto_hdr(key, value):
    """Bytes of one header entry (the role of PRESTO's sigproc.addto_hdr,
    bin/zero_dm_filter.py:26)."""
    if key in FLAG_KEYS:
        return _pack_string(key)
    if key in INT_KEYS:
        return _pack_string(key) + struct.pack("<i", int(value))
    if key in DOUBLE_KEYS:
        return _pack_string(key) + struct.pack("<d", float(value))
    if key in STRING_KEYS:
        return _pack_string(key) + _pack_string(str(value))
    if key in BYTE_KEYS:
        return _pack_string(key) + struct.pack("<b", int(value))
    raise ValueError("unknown SIGPROC header keyword %r" % key)


def read_header(f):
    """(header dict, ordered keyword list, header size in bytes) of an open
    filterbank file positioned at its start."""
    params, header = [], {}
    key = ""
    while key != "HEADER_END":
        key, val = read_hdr_val(f)
        header[key] = val
        params.append(key)
    return header, params, f.tell()


def write_header(f, header_params, header):
    """Write every keyword of ``header_params`` in order
    (bin/zero_dm_filter.py:21-27)."""
    for key in header_params:
        f.write(addto_hdr(key, header.get(key)))


def make_header(nchans, nbits, tsamp, fch1, foff, tstart=60000.0, source_name="synthetic",
                telescope_id=0, machine_id=0, src_raj=0.0, src_dej=0.0, nifs=1):
    """(header_params, header) of a minimal valid filterbank header."""
    header = dict(HEADER_START=None, telescope_id=telescope_id, machine_id=machine_id,
                  data_type=1, source_name=source_name, src_raj=src_raj, src_dej=src_dej,
                  tstart=tstart, tsamp=tsamp, nbits=nbits, fch1=fch1, foff=foff,
                  nchans=nchans, nifs=nifs, HEADER_END=None)
    params = ["HEADER_START", "telescope_id", "machine_id", "data_type", "source_name",
              "src_raj", "src_dej", "tstart", "tsamp", "nbits", "fch1", "foff", "nchans",
              "nifs", "HEADER_END"]
    return params, header
