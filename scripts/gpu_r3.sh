#!/bin/bash
# Round-3 GPU run: smoke, the GPU suite, the default bench line (configs[3],
# PCIe-inclusive leg + CPU baseline), the 8-rank rehearsal and both configs[4]
# zero-DM lines.  STAGES (default "tests bench"): any of tests bench rehearse
# stream.  Every GPU step has its own time limit; the first failure ends it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r3
mkdir -p $O
STAGES=${STAGES:-"tests bench"}
for s in $STAGES; do
  case $s in
    tests)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -5 $O/smoke.log; exit 1; }
      echo SMOKE_OK
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${TESTK:+-k "$TESTK"} > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
      tail -1 $O/pytest_gpu.log ;;
    bench)
      timeout -k 10 600 python bench.py > $O/bench_config3.json 2> $O/bench_config3.err || { echo BENCH_FAIL; tail -5 $O/bench_config3.err; exit 1; }
      cut -c1-400 $O/bench_config3.json ;;
    rehearse)
      timeout -k 10 600 python bench.py --rehearse 8 > $O/rehearse8.json 2> $O/rehearse8.err || { echo REHEARSE_FAIL; tail -5 $O/rehearse8.err; exit 1; }
      cut -c1-600 $O/rehearse8.json ;;
    stream)
      for z in wrap int; do
        timeout -k 10 300 python bench.py --config stream --zdm $z > $O/bench_stream_$z.json 2> $O/bench_stream_$z.err || { echo STREAM_FAIL $z; tail -5 $O/bench_stream_$z.err; exit 1; }
        cut -c1-300 $O/bench_stream_$z.json
      done ;;
  esac
done
