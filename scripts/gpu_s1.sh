#!/bin/bash
# Stage-1 A/B on one MI355X: the factorised parity tests (pattern-image
# poison on), then rocprofv3 kernel stats of bench.py for each config in CFGS.
#   O=gpurun_out/<dir> CFGS="config2 config3" TF="tests/..." bash scripts/gpu_s1.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=${O:-gpurun_out/s1}
mkdir -p $O
if [ -n "${TF-tests/test_gpu_factor.py}" ]; then
  timeout -k 10 600 python -u -m pytest ${TF-tests/test_gpu_factor.py} -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
for c in ${CFGS:-config2 config3}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt_$c -o kt --output-format csv -- python bench.py --config $c --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline --no-e2e > $O/kt_$c.log 2>&1 || { echo "kt $c failed"; tail -5 $O/kt_$c.log; exit 1; }
  python - $O/kt_$c/kt_kernel_stats.csv $c <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "pdd" in r["Name"]:
        print(sys.argv[2], r["Name"][:56], r["Calls"], "%.3f ms" % (float(r["AverageNs"]) / 1e6))
PY
done
