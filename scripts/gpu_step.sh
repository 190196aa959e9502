#!/bin/bash
# One development step on the GPU: the -m gpu suite, then production kernel
# times for configs[3] / configs[1] f32 / configs[1] u8, then the staging-alone
# decomposition point (dev build, dbg 2) for configs[3].
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/step
mkdir -p $O
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
k() { python -c "import json;d=json.load(open('$1'));r=d['roofline'];print('%.2f ms/launch x %g, value %.4g, frac %.4f' % (r['kernel_ms_per_launch'], r['launches_per_step'], d['value'], r['frac']))"; }
# BENCHES: config:args items, args comma-separated
for spec in ${BENCHES:-config3: config2:--dtype,f32 config2:--dtype,u8 northstar:}; do
  c=${spec%%:*}; a=${spec#*:}; a=${a//,/ }; n=$c$(echo $a | tr -d ' -')
  timeout -k 10 300 python bench.py --config $c $a --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $O/b_$n.json 2> $O/b_$n.err || { echo "bench $n failed"; tail -3 $O/b_$n.err; exit 1; }
  echo "$n: $(k $O/b_$n.json)"
done
for dbg in ${DBGS:-2}; do
  PDD_DEV_LIB=build/libpdd_dev.so PDD_SWEEP_DEBUG=$dbg timeout -k 10 300 python bench.py --config config3 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $O/d_$dbg.json 2> $O/d_$dbg.err || { echo "dev dbg $dbg failed"; tail -3 $O/d_$dbg.err; exit 1; }
  echo "config3 dev dbg=$dbg: $(k $O/d_$dbg.json)"
done
