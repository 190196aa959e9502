#!/bin/bash
# Round 6: stage-2 time decomposition + per-wave stamps of the developer
# build (build/libpdd_dev.so: PDD_SWEEP_DEBUG 1 = no window staging, 2 = no
# reads/adds, 4 = stamps) on the north star and configs[3].
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=${O:-gpurun_out/r6d}; mkdir -p $O
export PDD_DEV_LIB=build/libpdd_dev.so
for k in ns u8; do
  PDD_SWEEP_DEBUG=4 timeout -k 10 300 python scripts/probes/il_stamps.py $k > $O/stamps_$k.txt 2>&1 || { echo "stamps $k failed"; tail -5 $O/stamps_$k.txt; exit 1; }
  cat $O/stamps_$k.txt
done
for c in northstar config3; do
  for dbg in 0 1 2 3; do
    PDD_SWEEP_DEBUG=$dbg timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_${dbg}_$c -o kt --output-format csv -- python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $O/kt_${dbg}_$c.log 2>&1 || { echo "kt $dbg $c failed"; tail -5 $O/kt_${dbg}_$c.log; exit 1; }
    f=$(find $O/kt_${dbg}_$c -name "*kernel_stats.csv" | head -1)
    python - "$f" $dbg $c <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_sweep_il" in r["Name"]:
        print("dbg %s %-10s %9.3f ms" % (sys.argv[2], sys.argv[3], float(r["AverageNs"]) / 1e6))
PY
  done
done
