#!/bin/bash
# Round-4 stage-2 probes: per-wave stamps (dev build, PDD_SWEEP_DEBUG=4) of the
# factorised configs[3] / north-star tiles, the staging-form A/B (PDD_FX_STAGE)
# and the timing-only decomposition (devdma build).
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/r4probe; mkdir -p $O
for p in ${STAMPS:-"u8:3" "u8:11" "ns:3"}; do
  IFS=: read kind st <<< "$p"
  PDD_DEV_LIB=build/libpdd_dev.so PDD_SWEEP_DEBUG=4 PDD_FX_STAGE=$st timeout -k 10 120 python scripts/probes/il_stamps.py $kind > $O/stamps_${kind}_$st.txt 2>&1 || { echo "stamps $p failed"; tail -3 $O/stamps_${kind}_$st.txt; exit 1; }
  echo "stamps $p done"
done
if [ -n "$RUNS" ]; then RUNS="$RUNS" RUNT="${RUNT:-}" TF=tests/test_gpu_factor.py TK=factor bash scripts/gpu_fxstage.sh || exit 1; fi
if [ -n "$DBGS" ]; then LIBS=devdma DBGS="$DBGS" CFGS="${CFGS:-config3}" bash scripts/gpu_decomp.sh || exit 1; fi
if [ -n "$S1" ]; then
  for nt in $S1; do
    PDD_DEV_LIB=build/libpdd_dev.so PDD_FX_S1_NT=$nt timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_s1_$nt -o kt --output-format csv -- python bench.py --config config3 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $O/kt_s1_$nt.log 2>&1 || { echo "kt s1 $nt failed"; tail -3 $O/kt_s1_$nt.log; exit 1; }
    python - $O/kt_s1_$nt <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_fx" in r["Name"] or "k_sweep" in r["Name"]:
            print(sys.argv[1].split("/")[-1], r["Name"].split("(")[0][:70], r["Calls"], float(r["AverageNs"]) / 1e6)
PY
  done
fi
