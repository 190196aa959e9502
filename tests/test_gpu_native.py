"""The C-ABI driver (tests/native/abi_asan.cpp, built by __graft_entry__.build()
against pypulsar_amd/libpdd.so): argument checks, random sweep grids through
every tiling rung checked against a host sum, single-DM ops (corner turn,
shift + group sum with the sliced-partials path, exact integer zero-DM +
downsample, global statistics) against host loops, grouped plans and timing
pools, called straight through include/pdd.h with no Python in between.  It is the
regression test for library scratch reuse across calls: with stream-ordered
hipMallocAsync/hipFreeAsync images, a sequence of plan/execute/free calls
produced wrong planes (pool pages released at device synchronisation aliased
live buffers); the per-stream scratch arena fixed it."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "build", "abi_driver")

pytestmark = pytest.mark.gpu


def test_c_abi_driver(gpu):
    assert os.path.exists(DRIVER), "build/abi_driver missing: run __graft_entry__.build()"
    # (the driver poisons every factorised plan's pattern image through
    # pdd_sweep_plan_set_poison, see tests/test_gpu_factor.py)
    r = subprocess.run([DRIVER], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "0 failures" in r.stdout
