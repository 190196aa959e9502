"""The C ABI library loads and exports every symbol include/pdd.h declares.
CPU only: no compute call is made (there is no GPU here)."""
import os
import re

from conftest import ROOT


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "pdd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pdd_[a-z0-9_]+)\s*\(", src)))


def test_build_and_exports():
    import __graft_entry__ as g
    g.build()
    from pypulsar_amd import _lib
    h = _lib.lib()
    decl = declared_symbols()
    assert len(decl) >= 14
    for name in decl:
        assert hasattr(h, name), name
    assert sorted(_lib.EXPORTS) == decl
    assert h.pdd_version() >= 1


def test_error_path_without_gpu():
    # argument validation happens before any HIP call: a null pointer is
    # reported through pdd_last_error with a negative status
    import __graft_entry__ as g
    g.build()
    from pypulsar_amd import _lib
    h = _lib.lib()
    st = h.pdd_shift_pad(None, 4, 4, 4, None, 0, None, None, 4, 4, None)
    assert st < 0
    assert b"null pointer" in h.pdd_last_error()


def test_product_has_no_oracle_import():
    # the product package must never import the oracle (test infrastructure)
    pkg = os.path.join(ROOT, "pypulsar_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith(".py"):
                txt = open(os.path.join(dp, f)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle", txt, re.M), f
                assert "spectra_oracle" not in txt, f


def test_stale_library_refused(tmp_path):
    """The library carries the digest of the sources + flags it was built
    from (pdd_source_digest); a copy whose stamp differs from this tree is
    refused by the loader and would be rebuilt by build() -- so no stale
    binary (and no counters measured on one) passes for the current build."""
    import shutil
    import pytest
    import __graft_entry__ as g
    g.build()
    from pypulsar_amd import _digest, _lib
    want = _digest.source_digest()
    assert _digest.file_digest(g.LIB) == want
    assert not g.needs_build(g.LIB)
    assert _lib.open_library(g.LIB).pdd_source_digest().decode() == want
    stale = tmp_path / "libpdd_stale.so"
    shutil.copy(g.LIB, stale)
    data = bytearray(stale.read_bytes())
    i = data.find(_digest.MARKER) + len(_digest.MARKER)
    data[i:i + 16] = b"0123456789abcdef"
    stale.write_bytes(bytes(data))
    assert _digest.file_digest(str(stale)) == "0123456789abcdef"
    assert g.needs_build(str(stale))
    with pytest.raises(_lib.PddStaleLibrary):
        _lib.open_library(str(stale))


def test_library_reads_no_environment():
    """The production library takes its test switches through the C ABI
    (pdd_sweep_plan_set_poison / _set_segment_bytes): the only getenv calls
    in the sources are the developer knobs compiled under PDD_SWEEP_DEV."""
    csrc = os.path.join(ROOT, "pypulsar_amd", "csrc")
    for n in sorted(os.listdir(csrc)):
        if not n.endswith((".hip", ".h")):
            continue
        src = open(os.path.join(csrc, n)).read()
        dev = re.findall(r"#ifdef PDD_SWEEP_DEV(.*?)#else", src, flags=re.S)
        rest = src
        for d in dev:
            rest = rest.replace(d, "")
        assert "getenv" not in rest, n
