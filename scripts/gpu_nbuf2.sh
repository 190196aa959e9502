#!/bin/bash
# NBUF sweep of the u16 tiling in the dev build: production (dbg 0) and
# staging-alone (dbg 2), configs[3]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/nbuf2
mkdir -p $O
k() { python -c "import json;d=json.load(open('$1'));r=d['roofline'];print('%.2f ms/launch x %g' % (r['kernel_ms_per_launch'], r['launches_per_step']))"; }
for nb in ${NBUFS:-2 3 4}; do for dbg in ${DBGS:-0 2}; do
  PDD_SWEEP_NBUF=$nb PDD_DEV_LIB=build/libpdd_dev.so PDD_SWEEP_DEBUG=$dbg timeout -k 10 300 python bench.py --config ${CFG:-config3} --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $O/b_${nb}_$dbg.json 2> $O/b_${nb}_$dbg.err || { echo "nbuf $nb dbg $dbg failed"; tail -3 $O/b_${nb}_$dbg.err; exit 1; }
  echo "nbuf=$nb dbg=$dbg $(k $O/b_${nb}_$dbg.json)"
done; done
