#!/bin/bash
# Quick GPU iteration: build, sweep parity tests, one bench line per dtype.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
python -c "import __graft_entry__ as g; g.build()" \
 && timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "sweep or smoke" > gpurun_out/pytest_quick.log 2>&1 \
 && echo PYTEST_OK \
 && timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_f32.log 2>&1 \
 && timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --dtype u8 > gpurun_out/bench_u8.log 2>&1 \
 && echo BENCH_OK
rc=$?
tail -5 gpurun_out/pytest_quick.log
for f in gpurun_out/bench_f32.log gpurun_out/bench_u8.log; do [ -f $f ] && python -c "
import json,sys
l=[x for x in open('$f') if x.startswith('{')]
if l:
  d=json.loads(l[-1]); r=d['roofline']; print('$f', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], 'TF %.2f frac %.3f'%(r['achieved'], r['frac']), d['config']['plan'])
else: print(open('$f').read()[-2000:])
"; done
exit $rc
