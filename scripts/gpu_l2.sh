#!/bin/bash
# L2 hit rate and fabric fetch of the sweep kernel, plain vs persistent grid.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/l2
mkdir -p $O
for ps in 0 1; do
  PDD_SWEEP_PERSIST=$ps timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/hit_p$ps -o p --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCHX:-} > $O/hit_p$ps.log 2>&1 || { echo "pmc failed"; tail -5 $O/hit_p$ps.log; exit 1; }
  PDD_SWEEP_PERSIST=$ps timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_p$ps -o p --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCHX:-} > $O/fetch_p$ps.log 2>&1 || { echo "pmc failed"; tail -5 $O/fetch_p$ps.log; exit 1; }
done
python - <<'PY'
import csv, glob, collections
for ps in (0, 1):
    for tag in ("hit", "fetch"):
        acc = collections.defaultdict(lambda: collections.defaultdict(float))
        for f in glob.glob("gpurun_out/l2/%s_p%d/**/*counter_collection.csv" % (tag, ps), recursive=True):
            for r in csv.DictReader(open(f)):
                if "k_sweep_il" in r["Kernel_Name"]:
                    acc[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        for d, v in list(acc.items())[-1:]:
            print("persist", ps, tag, dict(v), ("hit %.3f" % (v["TCC_HIT_sum"] / (v["TCC_HIT_sum"] + v["TCC_MISS_sum"]))) if tag == "hit" else "")
PY
