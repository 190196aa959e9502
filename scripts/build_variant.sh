#!/bin/bash
# Tuning build of the working tree's production libpdd with extra defines
# (PDD_FX_GT, PDD_FX_PAIR_MAX, ...) into build/libpdd_<name>.so, loaded with
# PDD_DEV_LIB=build/libpdd_<name>.so:  scripts/build_variant.sh <name> [-DFOO=1 ...]
# (developer knobs -- stamps, timing-only decompositions: scripts/build_dev.sh)
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p build
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -fno-slp-vectorize \
  -ffp-contract=off "$@" -o build/libpdd_$name.so \
  pypulsar_amd/csrc/pdd_ops.hip pypulsar_amd/csrc/pdd_sweep.hip pypulsar_amd/csrc/pdd_search.hip \
  pypulsar_amd/csrc/pdd_psrfits.hip
