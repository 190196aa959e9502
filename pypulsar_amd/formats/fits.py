"""Minimal FITS reader/writer for PSRFITS search-mode files (primary HDU +
BINTABLE extensions), replacing ``astropy.io.fits`` (absent in this image)
for what ``formats/psrfits.py`` uses of it: ``open(fn)[name].header`` cards,
``.columns.names`` / ``.columns[i].format``, and row access
``.data[row][column]`` on a memory-mapped table.

FITS layout (FITS standard 4.0): every HDU is a header of 80-character
ASCII cards in 2880-byte blocks, closed by ``END``, followed by its data
padded to 2880 bytes.  A BINTABLE's data is NAXIS2 rows of NAXIS1 bytes;
column n has TTYPEn (name) and TFORMn (``rT``: repeat r of type T), stored
big-endian.  Heap (variable-length P/Q) columns are not supported.
"""
import builtins
import collections
import os

import numpy as np

BLOCK = 2880
CARD = 80

# TFORM type code -> (numpy big-endian base dtype, bytes per element)
_TFORM = {
    "L": ("S1", 1), "B": ("u1", 1), "I": (">i2", 2), "J": (">i4", 4), "K": (">i8", 8),
    "E": (">f4", 4), "D": (">f8", 8), "C": (">c8", 8), "M": (">c16", 16),
}


def _parse_value(v):
    v = v.strip()
    if not v:
        return None
    if v.startswith("'"):
        # string: '' is an escaped quote; trailing blanks are not significant
        out, i = [], 1
        while i < len(v):
            if v[i] == "'":
                if i + 1 < len(v) and v[i + 1] == "'":
                    out.append("'")
                    i += 2
                    continue
                break
            out.append(v[i])
            i += 1
        return "".join(out).rstrip()
    v = v.split("/", 1)[0].strip()
    if v == "T":
        return True
    if v == "F":
        return False
    try:
        return int(v)
    except ValueError:
        pass
    try:
        return float(v.replace("D", "E").replace("d", "e"))
    except ValueError:
        return v


class Header(collections.OrderedDict):
    """Keyword -> value (COMMENT / HISTORY cards dropped)."""

    def keys(self):  # noqa: D401  (astropy-style list of keys)
        return list(super().keys())


def read_header(f, offset):
    """Parse the header at byte ``offset``; returns (Header, header bytes)."""
    f.seek(offset)
    hdr = Header()
    nbytes = 0
    while True:
        block = f.read(BLOCK)
        if len(block) < BLOCK:
            raise ValueError("truncated FITS header at byte %d" % (offset + nbytes))
        nbytes += BLOCK
        for i in range(0, BLOCK, CARD):
            card = block[i:i + CARD].decode("ascii", "replace")
            key = card[:8].strip()
            if key == "END":
                return hdr, nbytes
            if key in ("", "COMMENT", "HISTORY") or card[8:10] != "= ":
                continue
            hdr[key] = _parse_value(card[10:])


class Column(object):
    def __init__(self, name, fmt, offset):
        self.name = name
        self.format = fmt
        self.offset = offset
        code = fmt.strip()
        i = 0
        while i < len(code) and code[i].isdigit():
            i += 1
        self.repeat = int(code[:i]) if i else 1
        self.code = code[i:i + 1]
        if self.code == "A":
            self.dtype, self.nbytes = "S%d" % self.repeat, self.repeat
        elif self.code == "X":
            self.dtype, self.nbytes = "u1", (self.repeat + 7) // 8
        elif self.code in _TFORM:
            base, size = _TFORM[self.code]
            self.dtype, self.nbytes = base, size * self.repeat
        else:
            raise ValueError("unsupported TFORM %r (column %s)" % (fmt, name))

    def np_field(self):
        if self.code in ("A",):
            return (self.name, self.dtype)
        n = self.repeat if self.code != "X" else self.nbytes
        return (self.name, self.dtype, (n,)) if n != 1 else (self.name, self.dtype)


class Columns(list):
    @property
    def names(self):
        return [c.name for c in self]


class HDU(object):
    def __init__(self, fn, header, data_offset):
        self.filename = fn
        self.header = header
        self.data_offset = data_offset
        self.name = header.get("EXTNAME", "PRIMARY") if "XTENSION" in header else "PRIMARY"
        bitpix = abs(int(header.get("BITPIX", 8)))
        naxis = int(header.get("NAXIS", 0))
        dims = [int(header["NAXIS%d" % (i + 1)]) for i in range(naxis)]
        n = int(np.prod(dims)) if dims else 0
        gcount = int(header.get("GCOUNT", 1))
        pcount = int(header.get("PCOUNT", 0))
        self.data_size = bitpix // 8 * gcount * (pcount + n) if naxis else 0
        self._data = None
        self.columns = Columns()
        if header.get("XTENSION") == "BINTABLE":
            off = 0
            for i in range(int(header.get("TFIELDS", 0))):
                col = Column(header.get("TTYPE%d" % (i + 1), "col%d" % (i + 1)),
                             header["TFORM%d" % (i + 1)], off)
                off += col.nbytes
                self.columns.append(col)
            if off != int(header["NAXIS1"]):
                raise ValueError("BINTABLE %s: columns span %d bytes, NAXIS1 is %d"
                                 % (self.name, off, header["NAXIS1"]))

    @property
    def data(self):
        """Structured memmap of the table rows (BINTABLE) or None."""
        if self._data is None and self.columns:
            dt = np.dtype([c.np_field() for c in self.columns])
            rows = int(self.header["NAXIS2"])
            self._data = np.memmap(self.filename, dtype=dt, mode="r", offset=self.data_offset,
                                   shape=(rows,)) if rows else np.zeros(0, dtype=dt)
        return self._data

    def raw_rows(self, lo, hi):
        """Bytes of rows [lo, hi) as a uint8 [hi-lo, NAXIS1] memmap view."""
        w = int(self.header["NAXIS1"])
        mm = np.memmap(self.filename, dtype=np.uint8, mode="r",
                       offset=self.data_offset + lo * w, shape=((hi - lo) * w,))
        return mm.reshape(hi - lo, w)


class FitsFile(list):
    """``open(fn)`` -> list of HDUs, indexable by position or EXTNAME."""

    def __init__(self, fn):
        super().__init__()
        self.filename = fn
        size = os.path.getsize(fn)
        with builtins.open(fn, "rb") as f:
            off = 0
            while off < size:
                hdr, hb = read_header(f, off)
                h = HDU(fn, hdr, off + hb)
                self.append(h)
                off += hb + -(-h.data_size // BLOCK) * BLOCK

    def __getitem__(self, key):
        if isinstance(key, str):
            for h in self:
                if h.name == key:
                    return h
            raise KeyError(key)
        return list.__getitem__(self, key)

    def close(self):
        pass


def open(fn, mode="readonly", memmap=True):  # noqa: A001  (astropy.io.fits.open)
    return FitsFile(fn)


# ----------------------------------------------------------------- writing
def _card(key, value, comment=None):
    if isinstance(value, bool):
        v = "%20s" % ("T" if value else "F")
    elif isinstance(value, (int, np.integer)):
        v = "%20d" % value
    elif isinstance(value, (float, np.floating)):
        v = "%20s" % repr(float(value)).upper()
    else:
        s = "'%-8s'" % str(value).replace("'", "''")
        v = "%-20s" % s
    c = "%-8s= %s" % (key, v)
    if comment:
        c += " / " + comment
    return c[:CARD].ljust(CARD)


def _header_bytes(cards):
    txt = "".join(_card(k, v) for k, v in cards) + "END".ljust(CARD)
    pad = -len(txt) % BLOCK
    return (txt + " " * pad).encode("ascii")


def write(fn, primary_cards, tables):
    """Write a primary HDU (no data) + BINTABLE extensions.

    ``tables``: list of (extname, header cards, columns, rows) where columns
    is [(name, tform)] and rows maps each column name to its per-row values
    (a dict of arrays or a structured array; any endianness, written
    big-endian)."""
    with builtins.open(fn, "wb") as f:
        cards = [("SIMPLE", True), ("BITPIX", 8), ("NAXIS", 0), ("EXTEND", True)]
        f.write(_header_bytes(cards + list(primary_cards)))
        for extname, hcards, columns, rows in tables:
            nrows = len(rows[columns[0][0]]) if columns else 0
            cols = [Column(n, t, 0) for n, t in columns]
            width = sum(c.nbytes for c in cols)
            cards = [("XTENSION", "BINTABLE"), ("BITPIX", 8), ("NAXIS", 2), ("NAXIS1", width),
                     ("NAXIS2", nrows), ("PCOUNT", 0), ("GCOUNT", 1),
                     ("TFIELDS", len(cols))]
            for i, (n, t) in enumerate(columns):
                cards += [("TTYPE%d" % (i + 1), n), ("TFORM%d" % (i + 1), t)]
            cards += [("EXTNAME", extname)] + list(hcards)
            f.write(_header_bytes(cards))
            dt = np.dtype([c.np_field() for c in cols])
            out = np.zeros(nrows, dtype=dt)
            for c in cols:
                out[c.name] = rows[c.name]
            b = out.tobytes()
            f.write(b + b"\0" * (-len(b) % BLOCK))
