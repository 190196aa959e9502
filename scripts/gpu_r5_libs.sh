#!/bin/bash
# Kernel ms per launch of developer libraries (build/libpdd_<lib>.so, loaded
# through PDD_DEV_LIB) for every config in CFGS and PDD_SWEEP_DEBUG value in
# DBGS (0 = production behaviour; 1 / 2 / 3 timing-only decompositions).
#   LIBS="a b" CFGS="config3 northstar" DBGS="0 3" O=gpurun_out/<dir>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=${O:-gpurun_out/libs}; mkdir -p $O
for c in ${CFGS:-config3 northstar}; do
  for dbg in ${DBGS:-0}; do
    for lib in ${LIBS}; do
      PDD_DEV_LIB=build/libpdd_$lib.so PDD_SWEEP_DEBUG=$dbg timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline --no-e2e > $O/b_${lib}_${c}_$dbg.json 2> $O/b_${lib}_${c}_$dbg.err || { echo "bench $lib $c $dbg failed"; tail -3 $O/b_${lib}_${c}_$dbg.err; exit 1; }
      echo "$c dbg=$dbg $lib $(python -c "import json;d=json.loads(open('$O/b_${lib}_${c}_$dbg.json').read().strip().splitlines()[-1]);r=d['roofline'];print('%.2f ms/launch x %s  step %.1f ms' % (r['kernel_ms_per_launch'], r['launches_per_step'], d['ms_per_step']))")"
    done
  done
done
