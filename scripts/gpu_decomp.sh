#!/bin/bash
# Time decomposition of k_sweep_il (dev build build/libpdd_dev.so, timing-only
# flags, wrong results): PDD_SWEEP_DEBUG 0 = production; 1 = loaders skip the
# window DMAs; 64 = no chunk barriers; 65 = neither; 2 = compute skips reads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/decomp
mkdir -p $O
for c in ${CFGS:-config3}; do
for lib in ${LIBS:-dev}; do
for dbg in ${DBGS:-0 1 64 65 2}; do
  PDD_DEV_LIB=build/libpdd_$lib.so PDD_SWEEP_DEBUG=$dbg timeout -k 10 300 python bench.py --config $c ${DTYPE:+--dtype $DTYPE} --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $O/b_${c}_$dbg.json 2> $O/b_${c}_$dbg.err || { echo "bench $c $dbg failed"; tail -3 $O/b_${c}_$dbg.err; exit 1; }
  echo "$c $lib dbg=$dbg $(python -c "import json;d=json.load(open('$O/b_${c}_$dbg.json'))['roofline'];print(d['kernel_ms_per_launch'], d['launches_per_step'])")"
done
done
done
