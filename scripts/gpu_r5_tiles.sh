#!/bin/bash
# Factorised stage 2 under tile-order variants (build/libpdd_<lib>.so built
# by scripts/build_variant.sh with -DPDD_FX_GT/GJ): kernel ms per launch
# from the bench's HIP events for every config in CFGS, and the sweep
# kernel's FETCH_SIZE (separate rocprofv3 --pmc pass) for the first config.
#   LIBS="t4x2 t8x2 ..." CFGS="config3 northstar" O=gpurun_out/<dir>
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=${O:-gpurun_out/tiles}; mkdir -p $O
CFGS=${CFGS:-config3 northstar}
first=${CFGS%% *}
for lib in ${LIBS:-t4x2}; do
  for c in $CFGS; do
    A="--config $c --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline --no-e2e"
    PDD_DEV_LIB=build/libpdd_$lib.so timeout -k 10 300 python bench.py $A > $O/b_${lib}_$c.json 2> $O/b_${lib}_$c.err || { echo "bench $lib $c failed"; tail -3 $O/b_${lib}_$c.err; exit 1; }
  done
  if [ -z "$NOFETCH" ]; then
    PDD_DEV_LIB=build/libpdd_$lib.so timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/fe_$lib -o p --output-format csv -- python bench.py --config $first --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $O/fe_$lib.log 2>&1 || { echo "fetch $lib failed"; tail -3 $O/fe_$lib.log; exit 1; }
  fi
  python - $O $lib "$CFGS" <<'PY'
import csv, glob, json, sys, collections
O, lib, cfgs = sys.argv[1], sys.argv[2], sys.argv[3].split()
fe = collections.defaultdict(float)
for f in glob.glob("%s/fe_%s/**/*counter_collection.csv" % (O, lib), recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == "FETCH_SIZE" and "k_sweep_il" in r["Kernel_Name"]:
            fe[r["Dispatch_Id"]] += float(r["Counter_Value"])
per = 2 * sum(fe.values()) / max(1, len(fe)) * 1024 / 1e9
out = []
for c in cfgs:
    d = json.loads(open("%s/b_%s_%s.json" % (O, lib, c)).read().strip().splitlines()[-1])
    out.append("%s %.2f ms/launch (step %.1f)" % (c, d["roofline"]["kernel_ms_per_launch"], d["ms_per_step"]))
print("%-6s %s  fetch(%s) %.1f GB/launch" % (lib, "  ".join(out), cfgs[0], per))
PY
done
