#!/bin/bash
# Developer build of libpdd with the PDD_SWEEP_DEV knobs (PDD_SWEEP_DEBUG,
# PDD_SWEEP_VARIANT, PDD_FX_STAGE) into build/libpdd_dev.so (DEV_OUT to
# change; DEV_FLAGS adds defines, e.g. -DPDD_DMA_MODES=1 for the timing-only
# DMA modes); load it with PDD_DEV_LIB=build/libpdd_dev.so.  Never used by
# tests, smoke or bench.
set -e
cd "$(dirname "$0")/.."
mkdir -p build
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -fno-slp-vectorize \
  -ffp-contract=off -DPDD_SWEEP_DEV ${DEV_FLAGS:-} -o ${DEV_OUT:-build/libpdd_dev.so} \
  pypulsar_amd/csrc/pdd_ops.hip pypulsar_amd/csrc/pdd_sweep.hip pypulsar_amd/csrc/pdd_search.hip \
  pypulsar_amd/csrc/pdd_psrfits.hip
