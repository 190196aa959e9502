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
