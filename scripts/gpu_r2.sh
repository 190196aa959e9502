#!/bin/bash
# Round-2 GPU pass: smoke, GPU parity suite, default bench (configs[3]), and a
# rocprofv3 kernel trace + stats of the same bench command.
# STAGES (env): subset of "smoke tests bench prof" (default: all).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r2
mkdir -p $O
ST=${STAGES:-"smoke tests bench prof"}
PYT=${PYTEST_ARGS:-"tests -m gpu"}
BA=${BENCH_ARGS:-""}
run() { echo "== $1 $(date +%T)"; }
rc=0
for s in $ST; do
  case $s in
    smoke) run smoke; timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > $O/smoke.log 2>&1 || { rc=$?; break; } ;;
    tests) run tests; timeout -k 10 1000 python -u -m pytest $PYT -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { rc=$?; break; } ;;
    bench) run bench; timeout -k 10 600 python bench.py $BA > $O/bench.json 2> $O/bench.err || { rc=$?; break; } ;;
    prof) run prof; timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python bench.py $BA --steps 2 --warmup 1 --no-cpu-baseline > $O/kt.log 2>&1 || { rc=$?; break; } ;;
  esac
done
echo "rc=$rc"
tail -5 $O/pytest_gpu.log 2>/dev/null
cut -c1-1500 $O/bench.json 2>/dev/null
tail -3 $O/bench.err $O/kt.log 2>/dev/null
exit $rc
