#!/bin/bash
# GPU-box check: smoke, GPU parity tests, a short bench. Each GPU step has its
# own time limit and the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > gpurun_out/smoke.log 2>&1 \
 && echo SMOKE_OK \
 && timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 \
 && echo PYTEST_OK \
 && timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_short.log 2>&1 \
 && echo BENCH_OK
rc=$?
tail -3 gpurun_out/smoke.log; tail -15 gpurun_out/pytest_gpu.log 2>/dev/null; tail -3 gpurun_out/bench_short.log 2>/dev/null
exit $rc
