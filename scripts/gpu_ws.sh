#!/bin/bash
# Sweep-kernel experiments: parity on the sweep tests per forced variant
# (VARS), kernel time per variant, then SQ counters of variant SQVAR.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/ws
mkdir -p $O
python -c "import __graft_entry__ as g; g.build()" > $O/build.log 2>&1 || { tail $O/build.log; exit 1; }
for v in ${VARS:-0 1 2}; do
  PDD_SWEEP_VARIANT=$v timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "${TESTK:-sweep}" --timeout 120 --timeout-method thread > $O/pytest_v$v.log 2>&1 || { echo "PYTEST FAIL v$v"; tail -30 $O/pytest_v$v.log; exit 1; }
  echo "v$v: $(tail -1 $O/pytest_v$v.log)"
done
: > $O/variants.log
for dt in ${DTYPES:-f32}; do for v in ${VARS:-0 1 2}; do
  PDD_SWEEP_VARIANT=$v timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --dtype $dt ${BENCHX:-} > $O/v.json 2>&1 || { cat $O/v.json; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('$O/v.json') if l.startswith('{')][-1])
print('$dt v=$v', 'ms %.2f'%d['roofline']['kernel_ms'], 'Tadd/s %.2f'%d['roofline']['achieved'], d['config']['plan'])" >> $O/variants.log
done; done
cat $O/variants.log
[ -n "${NOSQ:-}" ] && exit 0
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"
P2="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VMEM"
for p in 1 2; do
  eval C=\$P$p
  PDD_SWEEP_VARIANT=${SQVAR:-0} timeout -s KILL 90 rocprofv3 --pmc $C -d $O/sq_p$p -o p --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCHX:-} > $O/sq_p$p.log 2>&1 || { echo "pmc pass $p failed"; tail -5 $O/sq_p$p.log; exit 1; }
done
python scripts/pmc_summary.py $O
