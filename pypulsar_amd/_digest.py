"""Identity of a libpdd.so build (no torch, no GPU: used by build() before
the library is loaded).

source_digest() hashes every input of the production build -- the HIP
sources and headers under pypulsar_amd/csrc (recursively), include/pdd.h and
the compile flags -- into 16 hex digits.  build() compiles it into the
library (-DPDD_SRC_DIGEST, returned by pdd_source_digest()) and rebuilds
whenever the stamp in the file differs from the sources; _lib.lib() refuses
a library whose stamp differs; bench.py reports PMC traffic only for entries
stamped with the LOADED library's digest."""
import hashlib
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(_HERE)
CSRC = os.path.join(_HERE, "csrc")
HEADER = os.path.join(ROOT, "include", "pdd.h")
SOURCES = ["pdd_ops.hip", "pdd_sweep.hip", "pdd_search.hip", "pdd_psrfits.hip"]
FLAGS = ["-O3", "--offload-arch=gfx950", "-std=c++17", "-fPIC", "-shared", "-fno-slp-vectorize",
         "-ffp-contract=off"]
MARKER = b"pdd-src-digest:"


def _inputs():
    files = []
    for d, _, names in os.walk(CSRC):
        for n in names:
            if n.endswith((".hip", ".h", ".inc")):
                files.append(os.path.join(d, n))
    return sorted(files) + [HEADER]


def source_digest(flags=None):
    """sha256 (first 16 hex digits) of the library's sources + flags."""
    h = hashlib.sha256()
    for p in _inputs():
        with open(p, "rb") as f:
            h.update(os.path.relpath(p, ROOT).encode() + b"\0" + f.read())
    h.update(b"flags\0" + " ".join(FLAGS if flags is None else flags).encode())
    return h.hexdigest()[:16]


def sources_present():
    return os.path.isdir(CSRC) and os.path.exists(HEADER)


def file_digest(path):
    """The digest stamped into a built library file (None: no stamp)."""
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(MARKER)
    if i < 0:
        return None
    j = i + len(MARKER)
    return data[j:j + 16].decode("ascii", "replace")
