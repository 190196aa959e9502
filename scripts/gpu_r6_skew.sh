#!/bin/bash
# Round 6: delay-aligned factorised tiles (fx_skew) -- parity tests, then the
# north star and configs[3] lines with and without skew on one box (A/B).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=${O:-gpurun_out/r6a}
mkdir -p $O
timeout -k 10 600 python -u -m pytest ${TFILES:-tests/test_gpu_factor.py} -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() { local n=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "FAIL $n"; tail -5 $O/$n.err; exit 1; }; python -c "import json,sys; d=json.load(open('$O/$n.json')); r=d.get('roofline') or {}; print('$n', d['value'], d['ms_per_step'], r.get('frac'), r.get('kernel_ms_per_launch'))"; }
for c in ${CONFS:-northstar config3}; do
  run ${c}_skew --config $c --no-cpu-baseline --no-e2e ${BARGS:-}
  run ${c}_noskew --config $c --no-cpu-baseline --no-e2e --no-skew ${BARGS:-}
done
