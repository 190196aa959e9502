#!/bin/bash
# Staging-depth experiment (dev build build/libpdd_dev.so): the u16 tiling at
# NBUF chunk buffers, production (dbg 0) and staging-alone (dbg 2: compute
# waves skip their reads and adds; wrong planes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/nbuf
mkdir -p $O
for nb in ${NBUFS:-2 3 4 6}; do
for dbg in ${DBGS:-0 2}; do
  PDD_SWEEP_NBUF=$nb PDD_DEV_LIB=build/libpdd_dev.so PDD_SWEEP_DEBUG=$dbg timeout -k 10 300 python bench.py --config ${CFG:-config3} --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $O/b_${nb}_$dbg.json 2> $O/b_${nb}_$dbg.err || { echo "bench nbuf $nb dbg $dbg failed"; tail -3 $O/b_${nb}_$dbg.err; exit 1; }
  echo "nbuf=$nb dbg=$dbg $(python -c "import json;d=json.load(open('$O/b_${nb}_$dbg.json'));r=d['roofline'];print(r['kernel_ms_per_launch'], r['launches_per_step'], d['config']['plan']['lds_bytes'])")"
done
done
