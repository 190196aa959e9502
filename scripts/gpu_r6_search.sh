#!/bin/bash
# Single-pulse search kernels: GPU tests, the search bench line and its
# rocprofv3 kernel stats (each step under its own time limit; stops at the
# first failure).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=${O:-gpurun_out/r6se}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_search.py -q -x --timeout 240 --timeout-method thread > $O/t.log 2>&1 || { echo TEST_FAIL; tail -20 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python bench.py --config search > $O/b.json 2> $O/b.err || { echo BENCH_FAIL; tail -5 $O/b.err; exit 1; }
cut -c1-300 $O/b.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python bench.py --config search --steps 3 --warmup 1 > $O/kt.log 2>&1 || { echo PROF_FAIL; tail -5 $O/kt.log; exit 1; }
echo PROF_OK
if [ -n "$PMC" ]; then
  timeout -s KILL 120 rocprofv3 --pmc $PMC -d $O/pmc -o p --output-format csv -- python bench.py --config search --steps 2 --warmup 1 > $O/pmc.log 2>&1 || { echo PMC_FAIL; tail -5 $O/pmc.log; exit 1; }
  echo PMC_OK
fi
