#!/bin/bash
# rocprofv3 kernel stats for a few bench configs (CFGL="name|args;...").
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/profq
mkdir -p $O
IFS=';' read -ra L <<< "${CFGL:-subband|--config subband;stream|--config stream}"
for item in "${L[@]}"; do
  name=${item%%|*}; args=${item#*|}
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt_$name -o kt --output-format csv -- python bench.py $args --steps 3 --warmup 1 --no-cpu-baseline > $O/kt_$name.log 2>&1 || { echo "kt $name failed"; tail -5 $O/kt_$name.log; exit 1; }
  f=$(find $O/kt_$name -name "kt_kernel_stats.csv" | head -1)
  echo "== $name"; python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print("%-70s calls %5s avg %9.3f ms total %9.2f ms" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6))
PY
done
