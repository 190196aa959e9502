#!/bin/bash
# Per-kernel average durations (rocprofv3 --kernel-trace --stats) of developer
# libraries (build/libpdd_<lib>.so through PDD_DEV_LIB) on bench configs.
#   LIBS="a b" CFGS="config3 northstar" O=gpurun_out/<dir> [EXTRA="--dtype f32"]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=${O:-gpurun_out/kstats}; mkdir -p $O
for c in ${CFGS:-config3}; do
  for lib in ${LIBS}; do
    PDD_DEV_LIB=build/libpdd_$lib.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_${lib}_$c -o kt --output-format csv -- python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-e2e $EXTRA > $O/kt_${lib}_$c.log 2>&1 || { echo "kt $lib $c failed"; tail -5 $O/kt_${lib}_$c.log; exit 1; }
    f=$(find $O/kt_${lib}_$c -name "*kernel_stats.csv" | head -1)
    python - "$f" $lib $c <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "pdd::" in r["Name"]:
        print("%-5s %-10s %-62s %4s %9.3f ms" % (sys.argv[2], sys.argv[3], r["Name"][:62], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
  done
done
