#!/bin/bash
# Staggered-groups experiment: timings of forced u16 tilings (dev build), then
# the u8 sweep tests with the staggered tiling forced.
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONDONTWRITEBYTECODE=1
CFGS="config3:u8 config2:u8" VARS="${VARS:-0 2 4}" bash scripts/gpu_variant_sweep.sh || exit 1
PDD_DEV_LIB=build/libpdd_dev.so PDD_SWEEP_VARIANT=${TV:-2} timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "u8 and not full_length and not ladder and not grouped and not chain and not ddplan" > gpurun_out/stag_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/stag_pytest.log; exit $rc
