#!/bin/bash
# End-of-round evidence, part 1: smoke, the whole GPU suite, every bench line
# (configs[3] default with the CPU baseline, then the other configs).  Part 2
# (profiles) is scripts/gpu_prof_r2.sh.  Each GPU step has its own time limit;
# the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/final
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > $O/smoke.log 2>&1 && echo SMOKE_OK \
 && timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo PYTEST_OK \
 && timeout -k 10 600 python bench.py > $O/bench_config3.json 2> $O/bench_config3.err && echo BENCH_OK \
 && timeout -k 10 300 python bench.py --config config2 --no-cpu-baseline > $O/bench_config2_f32.json 2> $O/e1 \
 && timeout -k 10 300 python bench.py --config config2 --dtype u8 --no-cpu-baseline > $O/bench_config2_u8.json 2> $O/e2 \
 && timeout -k 10 300 python bench.py --config northstar --no-cpu-baseline > $O/bench_northstar.json 2> $O/e3 \
 && timeout -k 10 300 python bench.py --config stream > $O/bench_stream.json 2> $O/e4 \
 && timeout -k 10 300 python bench.py --config subband > $O/bench_subband.json 2> $O/e5 \
 && timeout -k 10 300 python bench.py --config search > $O/bench_search.json 2> $O/e6 \
 && timeout -k 10 300 python bench.py --config ops > $O/bench_ops.json 2> $O/e7 && echo BENCHES_OK
rc=$?
tail -2 $O/pytest_gpu.log
for f in $O/bench_*.json; do echo "$f: $(cut -c1-200 $f)"; done
exit $rc
