#!/bin/bash
# Factorised staging forms (PDD_FX_STAGE 0 / 1, dev build) on the north star
# at groups of 2 and 4 and configs[3]; then the factor tests under each form.
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONDONTWRITEBYTECODE=1 PDD_DEV_LIB=build/libpdd_dev.so
O=gpurun_out/fxs; mkdir -p $O
k() { python -c "
import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline']
print('kernel %.2f ms  step %.1f ms  value %.3e' % (r['kernel_ms_per_launch'], d['ms_per_step'], d['value']))" $1; }
for run in "northstar 2 0" "northstar 2 1" "northstar 4 0" "northstar 4 1" "config3 4 0" "config3 4 1" "config3 2 1"; do
  set -- $run
  PDD_FX_STAGE=$3 timeout -k 10 200 python bench.py --config $1 --factor $2 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $O/b.json 2> $O/b.err || { echo "FAIL $run"; tail -3 $O/b.err; exit 1; }
  echo "$1 g=$2 stage=$3: $(k $O/b.json)"
done
for st in 1 0; do
  PDD_FX_STAGE=$st timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "factor or config or sweep" > $O/pytest_$st.log 2>&1
  rc=$?; echo "tests stage=$st: $(tail -1 $O/pytest_$st.log)"; [ $rc -eq 0 ] || exit $rc
done
