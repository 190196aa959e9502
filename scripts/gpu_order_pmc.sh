#!/bin/bash
# Tile-order experiment: FETCH_SIZE and kernel time of k_sweep_il for the
# default 2-D blocked order vs the XCD-contiguous order (PDD_SWEEP_DEBUG=16).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/order
A="--steps 3 --warmup 1 --no-cpu-baseline"
for dt in f32 u8; do
  for dbg in 0 16; do
    PDD_SWEEP_DEBUG=$dbg timeout -k 10 200 python bench.py $A --dtype $dt > gpurun_out/order/bench_${dt}_${dbg}.json 2>/dev/null || exit 1
    PDD_SWEEP_DEBUG=$dbg timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/order/pmc_${dt}_${dbg} -o p --output-format csv -- python bench.py $A --dtype $dt > gpurun_out/order/pmc_${dt}_${dbg}.log 2>&1 || exit 1
  done
done
python scripts/pmc_summary.py gpurun_out/order > gpurun_out/order/summary.txt
echo ORDER_OK
