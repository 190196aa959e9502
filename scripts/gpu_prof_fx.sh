#!/bin/bash
# rocprofv3 kernel stats of one bench line (CFG, ARGS) into gpurun_out/prof_<NAME>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
N=${NAME:-fx}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$N -o kt --output-format csv -- python bench.py --config ${CFG:-config3} ${ARGS} --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/prof_$N.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_$N.log; exit 1; }
f=$(find gpurun_out/prof_$N -name "*kernel_stats.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print("%-60s calls %6s  total %9.2f ms  avg %8.3f ms" % (r["Name"][:60], r["Calls"], float(r["TotalDurationNs"])/1e6, float(r["AverageNs"])/1e6))
PY
