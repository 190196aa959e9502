"""bench.py's PMC gate (load_pmc): a profiles/pmc_sweep.json entry is used
for the line's `traffic` only when it was measured on the LOADED library
(source digest), with the running plan and in the same run context (mode,
world size, launches per step).  Host logic only: the loaded digest is
stubbed."""
import importlib.util
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_pmc", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


PLAN = {"D": 4096, "C": 4096, "dms_per_block": 96, "samples_per_block": 1024, "lds_bytes": 160768,
        "max_bin": 14504, "min_bin": 0, "variant": 0}
CTX = {"mode": "dmshard", "world": 1, "launches_per_step": 4.0}


def _write(tmp_path, entry):
    p = tmp_path / "pmc_sweep.json"
    p.write_text(json.dumps({"config3_u8": entry}))
    return str(p)


def _entry(**kw):
    e = {"kernel": "k_sweep_il", "hbm_bytes_per_launch": 3.0e11, "src_digest": "abc123",
         "plan": PLAN, "ctx": CTX}
    e.update(kw)
    return e


def test_pmc_accepted_for_the_same_build_plan_and_run(bench, tmp_path, monkeypatch):
    from pypulsar_amd import _lib
    monkeypatch.setattr(_lib, "loaded_digest", lambda: "abc123")
    path = _write(tmp_path, _entry())
    got = bench.load_pmc(path, "config3_u8", PLAN, CTX)
    assert got is not None and got["hbm_bytes_per_launch"] == 3.0e11


@pytest.mark.parametrize("change", ["digest", "plan", "ctx", "key", "missing"])
def test_pmc_refused_otherwise(bench, tmp_path, monkeypatch, change):
    from pypulsar_amd import _lib
    monkeypatch.setattr(_lib, "loaded_digest", lambda: "abc123")
    entry = _entry()
    key = "config3_u8"
    if change == "digest":
        entry["src_digest"] = "stale00"
    elif change == "plan":
        entry["plan"] = dict(PLAN, dms_per_block=72)
    elif change == "ctx":
        entry["ctx"] = dict(CTX, mode="timeshard", world=8, launches_per_step=1.0)
    elif change == "key":
        key = "northstar"
    path = _write(tmp_path, entry) if change != "missing" else str(tmp_path / "absent.json")
    assert bench.load_pmc(path, key, PLAN, CTX) is None


def test_pmc_refused_when_the_library_cannot_report(bench, tmp_path, monkeypatch):
    from pypulsar_amd import _lib

    def boom():
        raise OSError("no library")
    monkeypatch.setattr(_lib, "loaded_digest", boom)
    assert bench.load_pmc(_write(tmp_path, _entry()), "config3_u8", PLAN, CTX) is None
