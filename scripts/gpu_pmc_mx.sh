#!/bin/bash
# PMC passes over scripts/probes/mx_pmc.py (dev build, PDD_SWEEP_DEBUG=$DBG).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/pmc_mx
mkdir -p $O
export PDD_DEV_LIB=build/libpdd_dev.so PDD_SWEEP_MX=${MX:-1} PDD_SWEEP_DEBUG=${DBG:-0}
i=0
for C in "SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_LDS_UNALIGNED_STALL" "FETCH_SIZE TA_BUSY_avr" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C -d $O/p$i -o p --output-format csv -- python scripts/probes/mx_pmc.py > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmc_mx/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-40:]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "sweep" not in k and "prep" not in k: continue
    print(k, {c: "%.4g" % (sum(v) / max(1, len(v)) * (1 if True else 1)) for c, v in d.items()})
PY
