#!/bin/bash
# Sweep-kernel experiments: candidate tilings, with and without restaging.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
python -c "import __graft_entry__ as g; g.build()" || exit 1
hipcc -O3 --offload-arch=gfx950 -o /tmp/glds_probe scripts/probes/glds_ubyte.hip && timeout -k 5 30 /tmp/glds_probe > gpurun_out/probe.log 2>&1; cat gpurun_out/probe.log
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "sweep or smoke or execute" > gpurun_out/pytest_quick.log 2>&1 || { tail -30 gpurun_out/pytest_quick.log; exit 1; }
tail -2 gpurun_out/pytest_quick.log
: > gpurun_out/variants.log
for dt in ${DTYPES:-f32 u8}; do for v in ${VARS:-0 1}; do for dbg in ${DBGS:-0 1}; do
  PDD_SWEEP_VARIANT=$v PDD_SWEEP_DEBUG=$dbg timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --dtype $dt > gpurun_out/v.json 2>&1 || { cat gpurun_out/v.json; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/v.json') if l.startswith('{')][-1])
print('$dt v=$v dbg=$dbg', 'ms %.2f'%d['roofline']['kernel_ms'], 'Tadd/s %.2f'%d['roofline']['achieved'], d['config']['plan'])" >> gpurun_out/variants.log
done; done; done
cat gpurun_out/variants.log
