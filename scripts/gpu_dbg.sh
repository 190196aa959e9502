#!/bin/bash
# Kernel time of the default sweep with the timing-only debug modes:
# PDD_SWEEP_DEBUG=1 skips the sample DMAs, =2 skips the compute.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/dbg
mkdir -p $O
python -c "import __graft_entry__ as g; g.build()" > $O/build.log 2>&1 || { tail $O/build.log; exit 1; }
for dt in ${DTYPES:-f32}; do for dbg in ${DBGS:-0 1 2 3}; do
  PDD_SWEEP_DEBUG=$dbg timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --dtype $dt ${BENCHX:-} > $O/v.json 2>&1 || { cat $O/v.json; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('$O/v.json') if l.startswith('{')][-1])
print('$dt dbg=$dbg', 'ms %.2f'%d['roofline']['kernel_ms'], 'Tadd/s %.2f'%d['roofline']['achieved'])"
done; done
