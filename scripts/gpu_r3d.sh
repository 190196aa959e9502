#!/bin/bash
# Session-3 check of the committed tree: smoke + the GPU suite on the in-tree
# library, then the default configs[3] line and the north-star line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r3d; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -5 $O/smoke.log; exit 1; }
echo SMOKE_OK
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python bench.py > $O/bench_config3.json 2> $O/bench_config3.err || { echo BENCH_FAIL; tail -5 $O/bench_config3.err; exit 1; }
cut -c1-400 $O/bench_config3.json
timeout -k 10 300 python bench.py --config northstar --no-cpu-baseline --no-e2e > $O/bench_northstar.json 2> $O/bench_northstar.err || { echo BENCH_FAIL; tail -5 $O/bench_northstar.err; exit 1; }
cut -c1-300 $O/bench_northstar.json
