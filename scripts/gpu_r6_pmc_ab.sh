#!/bin/bash
# Round 6: FETCH_SIZE of the factorised stage 2, delay-aligned vs plane-aligned
# tiles (bench.py --no-skew), configs[3] and the north star, one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=${O:-gpurun_out/r6k}; mkdir -p $O
for c in config3 northstar; do
  for v in skew noskew; do
    X=""; [ $v = noskew ] && X="--no-skew"
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/fe_${c}_$v -o p --output-format csv -- python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-e2e $X > $O/fe_${c}_$v.log 2>&1 || { echo "fetch $c $v failed"; tail -3 $O/fe_${c}_$v.log; exit 1; }
    f=$(find $O/fe_${c}_$v -name "*counter_collection.csv" | head -1)
    python - "$f" $c $v <<'PY'
import csv, sys, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if r["Counter_Name"] == "FETCH_SIZE" and "k_sweep_il" in r["Kernel_Name"]:
        acc[r["Dispatch_Id"]].append(float(r["Counter_Value"]))
v = [sum(x) for x in acc.values()]
print("%-10s %-7s k_sweep_il FETCH_SIZE x2 per launch: %.1f GB (%d launches)" % (sys.argv[2], sys.argv[3], 2 * 1024 * sum(v) / len(v) / 1e9, len(v)))
PY
  done
done
