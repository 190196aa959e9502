#!/bin/bash
# Factorised stage 2 under developer variants (build/libpdd_<lib>.so: tile
# orders -DPDD_IL_GT/GJ, DMA cache policy): kernel ms per launch from the
# bench's HIP events and the sweep kernel's FETCH_SIZE from a separate
# rocprofv3 --pmc pass.  LIBS="dev t1x32 ..." CFG=config3
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/tileorder; mkdir -p $O
C=${CFG:-config3}
for lib in ${LIBS:-dev}; do
  A="--config $C --steps 2 --warmup 1 --no-cpu-baseline --no-e2e"
  PDD_DEV_LIB=build/libpdd_$lib.so timeout -k 10 300 python bench.py $A > $O/b_$lib.json 2> $O/b_$lib.err || { echo "bench $lib failed"; tail -3 $O/b_$lib.err; exit 1; }
  PDD_DEV_LIB=build/libpdd_$lib.so timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/fe_$lib -o p --output-format csv -- python bench.py $A > $O/fe_$lib.log 2>&1 || { echo "fetch $lib failed"; tail -3 $O/fe_$lib.log; exit 1; }
  python - $O $lib <<'PY'
import csv, glob, json, sys, collections
O, lib = sys.argv[1], sys.argv[2]
d = json.load(open("%s/b_%s.json" % (O, lib)))
fe = collections.defaultdict(float); n = collections.defaultdict(set)
for f in glob.glob("%s/fe_%s/**/*counter_collection.csv" % (O, lib), recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == "FETCH_SIZE" and "k_sweep_il" in r["Kernel_Name"]:
            fe[r["Dispatch_Id"]] += float(r["Counter_Value"]); n[0].add(r["Dispatch_Id"])
per = 2 * sum(fe.values()) / max(1, len(fe)) * 1024 / 1e9
print("%-8s kernel %.2f ms  step %.1f ms  fetch %.1f GB/launch" % (lib, d["roofline"]["kernel_ms_per_launch"], d["ms_per_step"], per))
PY
done
