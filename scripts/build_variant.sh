#!/bin/bash
# Developer build of the working tree's libpdd with extra defines into
# build/libpdd_<name>.so:  scripts/build_variant.sh <name> [-DFOO=1 ...]
# (NODEV=1: without the PDD_SWEEP_DEV knobs, i.e. the production code)
set -e
cd "$(dirname "$0")/.."
name=$1; shift
dev=-DPDD_SWEEP_DEV; [ -n "$NODEV" ] && dev=
mkdir -p build
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -fno-slp-vectorize \
  -ffp-contract=off $dev "$@" -o build/libpdd_$name.so \
  pypulsar_amd/csrc/pdd_ops.hip pypulsar_amd/csrc/pdd_sweep.hip pypulsar_amd/csrc/pdd_search.hip \
  pypulsar_amd/csrc/pdd_psrfits.hip
