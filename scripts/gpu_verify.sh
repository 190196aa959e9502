#!/bin/bash
# Quick GPU-box verification of the tree: smoke, the GPU suite, the default
# bench line (configs[3]) and the configs[2] subband line.  Each GPU step has
# its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/verify
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > $O/smoke.log 2>&1 && echo SMOKE_OK \
 && timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo PYTEST_OK \
 && timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_config3.json 2> $O/e0 && echo BENCH_OK \
 && timeout -k 10 300 python bench.py --config subband --no-cpu-baseline > $O/bench_subband.json 2> $O/e1 && echo SUBBAND_OK
rc=$?
tail -3 $O/pytest_gpu.log
for f in $O/bench_*.json; do echo "$f: $(cut -c1-400 $f)"; done
exit $rc
