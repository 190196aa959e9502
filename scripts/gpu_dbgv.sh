#!/bin/bash
# Kernel time per (variant, debug flags) pair: PAIRS="v:dbg v:dbg ..."
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/dbgv
mkdir -p $O
python -c "import __graft_entry__ as g; g.build()" > $O/build.log 2>&1 || { tail $O/build.log; exit 1; }
for pr in ${PAIRS:-0:0}; do
  v=${pr%%:*}; dbg=${pr##*:}
  PDD_SWEEP_VARIANT=$v PDD_SWEEP_DEBUG=$dbg timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --dtype ${DT:-f32} ${BENCHX:-} > $O/v.json 2>&1 || { cat $O/v.json; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('$O/v.json') if l.startswith('{')][-1])
print('v=$v dbg=$dbg', 'ms %.2f'%d['roofline']['kernel_ms'], 'Tadd/s %.2f'%d['roofline']['achieved'])"
done
