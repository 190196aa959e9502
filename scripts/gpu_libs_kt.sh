#!/bin/bash
# rocprofv3 kernel stats of one bench config per library (dev A/B):
#   LIBS="fxe512 fxe1024" CFGS="config2 config3" O=gpurun_out/x bash scripts/gpu_libs_kt.sh
# (PDD_DEV_LIB=build/libpdd_<lib>.so; never the tests, smoke or bench defaults)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=${O:-gpurun_out/libs_kt}
mkdir -p $O
for c in ${CFGS:-config2}; do
for lib in ${LIBS:-fxe512}; do
  d=$O/kt_${c}_$lib
  PDD_DEV_LIB=build/libpdd_$lib.so timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $d -o kt --output-format csv -- python bench.py --config $c --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-e2e > $d.log 2>&1 || { echo "kt $c $lib failed"; tail -5 $d.log; exit 1; }
  python - $d/kt_kernel_stats.csv "$c $lib" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "pdd" in r["Name"]:
        print(sys.argv[2], r["Name"][:48], r["Calls"], "%.3f ms" % (float(r["AverageNs"]) / 1e6))
PY
done
done
