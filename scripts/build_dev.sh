#!/bin/bash
# Developer build of libpdd with the developer knobs (PDD_SWEEP_DEBUG
# stamps / timing-only decompositions, PDD_SWEEP_VARIANT forced tilings, the
# planner's model printout) into build/libpdd_dev.so (DEV_OUT to change;
# DEV_FLAGS adds defines).  The knobs are not in the production source: they
# are scripts/probes/dev_knobs.patch, applied here to a copy of the sources
# under build/dev_src.  Load the result with PDD_DEV_LIB=build/libpdd_dev.so.
# Never used by tests, smoke or bench.
set -e
cd "$(dirname "$0")/.."
rm -rf build/dev_src && mkdir -p build/dev_src/pypulsar_amd && cp -r pypulsar_amd/csrc build/dev_src/pypulsar_amd/ && cp -r include build/dev_src/
(cd build/dev_src && patch -s -p1 < ../../scripts/probes/dev_knobs.patch)
S=build/dev_src/pypulsar_amd/csrc
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -fno-slp-vectorize \
  -ffp-contract=off -DPDD_SWEEP_DEV ${DEV_FLAGS:-} -I include -o ${DEV_OUT:-build/libpdd_dev.so} \
  $S/pdd_ops.hip $S/pdd_sweep.hip $S/pdd_search.hip $S/pdd_psrfits.hip
