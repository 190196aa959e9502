#!/bin/bash
# Developer A/B helper: builds HEAD's pdd_sweep.hip (with the working tree's
# other sources) into build/libpdd_base.so; load with PDD_DEV_LIB.
set -e
cd "$(dirname "$0")/.."
mkdir -p build
git show HEAD:pypulsar_amd/csrc/pdd_sweep.hip > build/pdd_sweep_base.hip
cp pypulsar_amd/csrc/*.h build/ 2>/dev/null || true
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -fno-slp-vectorize \
  -ffp-contract=off -DPDD_SWEEP_DEV -Ipypulsar_amd/csrc -Iinclude -o build/libpdd_base.so \
  pypulsar_amd/csrc/pdd_ops.hip build/pdd_sweep_base.hip pypulsar_amd/csrc/pdd_search.hip \
  pypulsar_amd/csrc/pdd_psrfits.hip
