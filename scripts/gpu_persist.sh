#!/bin/bash
# Persistent-grid / variant experiment: parity with PDD_SWEEP_PERSIST=0 and 1,
# then sweep-kernel time per (dtype, variant, persist).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/persist
mkdir -p $O
python -c "import __graft_entry__ as g; g.build()" > $O/build.log 2>&1 || { tail $O/build.log; exit 1; }
for ps in 0; do
  PDD_SWEEP_PERSIST=$ps timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "${TESTK:-sweep or grouped or stream or parity}" --timeout 120 --timeout-method thread > $O/pytest_p$ps.log 2>&1 || { echo "PYTEST FAIL persist=$ps"; tail -30 $O/pytest_p$ps.log; exit 1; }
  echo "persist=$ps: $(tail -1 $O/pytest_p$ps.log)"
done
: > $O/variants.log
for run in ${RUNS:-f32:0:0 f32:0:1 u8:0:0 u8:0:1 u8:1:1 u8:2:1 u8:3:1}; do
  IFS=: read dt v ps <<< "$run"
  PDD_SWEEP_PERSIST=$ps PDD_SWEEP_VARIANT=$v timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --dtype $dt > $O/v.json 2>&1 || { cat $O/v.json; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('$O/v.json') if l.startswith('{')][-1])
print('$dt v=$v persist=$ps', 'ms %.2f'%d['roofline']['kernel_ms'], 'Tadd/s %.2f'%d['roofline']['achieved'], 'step %.2f'%d['ms_per_step'])" >> $O/variants.log
done
cat $O/variants.log
