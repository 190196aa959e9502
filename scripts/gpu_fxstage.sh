#!/bin/bash
# Factorised staging forms (PDD_FX_STAGE 0 / 1 / 2, dev build) on configs[3]
# and the north star; then the GPU tests of the factor paths under RUNT forms.
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONDONTWRITEBYTECODE=1 PDD_DEV_LIB=build/libpdd_dev.so
O=gpurun_out/fxs; mkdir -p $O
k() { python -c "
import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline']
print('kernel %.2f ms  step %.1f ms  value %.3e' % (r['kernel_ms_per_launch'], d['ms_per_step'], d['value']))" $1; }
for run in ${RUNS-"config3:4:1" "config3:4:2" "northstar:2:0" "northstar:2:2" "northstar:4:2"}; do
  IFS=: read c g st var <<< "$run"
  PDD_SWEEP_VARIANT=${var:-0} PDD_FX_STAGE=$st timeout -k 10 200 python bench.py --config $c --factor $g --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $O/b.json 2> $O/b.err || { echo "FAIL $run"; tail -3 $O/b.err; exit 1; }
  echo "$c g=$g stage=$st variant=${var:-0}: $(k $O/b.json)"
done
for st in ${RUNT-2}; do
  PDD_SWEEP_VARIANT=${RUNV:-0} PDD_FX_STAGE=$st timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread ${TF:-tests} -k "${TK:-factor or config or sweep}" > $O/pytest_$st.log 2>&1
  rc=$?; echo "tests stage=$st: $(tail -1 $O/pytest_$st.log)"; [ $rc -eq 0 ] || exit $rc
done
