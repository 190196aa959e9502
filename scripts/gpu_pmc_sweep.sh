#!/bin/bash
# PMC passes (one rocprofv3 --pmc run each, no tracing) over one production
# 8-bit sweep launch pair at the configs[3] grid (scripts/probes/mx_pmc.py
# without the dev library): LDS/VALU issue counts, LDS-array cycles, waits and
# the GPU clock (GRBM_GUI_ACTIVE over the kernel duration).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/pmc_sw
mkdir -p $O
P=${PROBE:-scripts/probes/mx_pmc.py}
i=0
for C in "SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C -d $O/p$i -o p --output-format csv -- python $P > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python $P > $O/kt.log 2>&1 || { echo "kt failed"; exit 1; }
python - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmc_sw/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-48:]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in glob.glob("gpurun_out/pmc_sw/kt/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print("%-60s avg %.3f ms" % (r["Name"].split("(")[0][-48:], float(r["AverageNs"]) / 1e6))
for k, d in agg.items():
    if "sweep" not in k: continue
    print(k)
    for c, v in sorted(d.items()):
        print("   %-24s %.5g" % (c, sum(v) / len(v)))
PY
