#!/bin/bash
# Host-ASan build of libpdd + the C-ABI driver tests/native/abi_asan.cpp
# (host code instrumented; device code built normally for gfx950).  Build
# here, run on the GPU box:  scripts/asan_check.sh build | run
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
case "${1:-build}" in
  build)
    mkdir -p build
    /opt/rocm/bin/hipcc -O3 -g --offload-arch=gfx950 -std=c++17 -fno-slp-vectorize -ffp-contract=off \
      -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer \
      -Iinclude -Ipypulsar_amd/csrc -o build/abi_asan tests/native/abi_asan.cpp \
      pypulsar_amd/csrc/pdd_ops.hip pypulsar_amd/csrc/pdd_sweep.hip pypulsar_amd/csrc/pdd_search.hip \
      pypulsar_amd/csrc/pdd_psrfits.hip
    ;;
  run)
    set +e
    mkdir -p gpurun_out
    ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 timeout -k 10 300 ./build/abi_asan > gpurun_out/abi_asan.log 2>&1
    rc=$?; tail -20 gpurun_out/abi_asan.log; exit $rc
    ;;
esac
