#!/bin/bash
# LDS / issue / cache PMC passes (one rocprofv3 --pmc run each, no tracing)
# over the factorised sweep of scripts/probes/fx_pmc.py at the configs[3] and
# north-star grids, plus a kernel-trace pass for the durations.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=${O:-gpurun_out/pmc_lds}
mkdir -p $O
P=scripts/probes/fx_pmc.py
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
for G in ${GRIDS:-4096 2048}; do
  i=0
  while IFS= read -r CS; do
    [ -z "$CS" ] && continue
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $CS -d $O/g$G/p$i -o p --output-format csv -- python $P $G ${LOGN:-20} > $O/g$G.p$i.log 2>&1 || { echo "pass $G/$i failed"; tail -5 $O/g$G.p$i.log; exit 1; }
  done <<< "${PASSES:-SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM
TCC_HIT_sum TCC_MISS_sum
FETCH_SIZE}"
  timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/g$G/kt -o kt --output-format csv -- python $P $G ${LOGN:-20} > $O/g$G.kt.log 2>&1 || { echo "kt $G failed"; exit 1; }
  echo "grid $G ok"
done
python - <<'PY'
import csv, glob, collections, os
O = os.environ.get("O", "gpurun_out/pmc_lds")
for gdir in sorted(glob.glob(O + "/g*/")):
    print("==", gdir)
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(gdir + "p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"].split("(")[0][-60:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for f in glob.glob(gdir + "kt/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            print("  %-62s n %s avg %.3f ms" % (r["Name"].split("(")[0][-60:], r["Calls"], float(r["AverageNs"]) / 1e6))
    for k, d in agg.items():
        if "sweep" not in k and "fx_" not in k:
            continue
        print(" ", k)
        for c, v in sorted(d.items()):
            print("     %-24s %.5g" % (c, sum(v) / len(v)))
PY
