"""Host logic of the factorised-sweep options (no GPU): DMSweep(factor=...)
-> pdd_sweep_plan_create_ex flags (include/pdd.h PDD_SWEEP_FACTOR*), and the
bench --factor option."""
import re
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _flags(factor):
    from pypulsar_amd.sweep import DMSweep
    sw = DMSweep.__new__(DMSweep)  # no plan: only the option mapping
    if factor == "force":
        factor = "force4"
    sw.factor = factor
    return sw._factor_flags()


def test_flag_values_match_header():
    from pypulsar_amd import _lib
    src = open(os.path.join(ROOT, "include", "pdd.h")).read()
    for name, val in (("PDD_SWEEP_FACTOR", _lib.SWEEP_FACTOR),
                      ("PDD_SWEEP_FACTOR_FORCE", _lib.SWEEP_FACTOR_FORCE),
                      ("PDD_SWEEP_FACTOR_G2", _lib.SWEEP_FACTOR_G2),
                      ("PDD_SWEEP_FACTOR_G4", _lib.SWEEP_FACTOR_G4),
                      ("PDD_SWEEP_NO_SKEW", _lib.SWEEP_NO_SKEW)):
        m = re.search(r"#define %s (\d+)" % name, src)
        assert m and int(m.group(1)) == val, name


@pytest.mark.parametrize("factor,want", [
    (True, 1), (False, 0), (2, 1 | 4), (4, 1 | 8),
    ("force2", 1 | 2 | 4), ("force4", 1 | 2 | 8), ("force", 1 | 2 | 8)])
def test_dmsweep_factor_flags(factor, want):
    assert _flags(factor) == want


def test_bench_factor_option():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)

    class A(object):
        pass
    for opt, want in (("auto", True), ("off", False), ("2", 2), ("4", 4), ("force2", "force2"),
                      ("force4", "force4")):
        a = A()
        a.factor = opt
        assert bench._factor_arg(a) == want
